# section stamps at HEAD (Cornell, config 4)
set -u
cd $GRAFT_REPO_ROOT
bash scripts/stamps.sh "cornell||" "sphere||--scene sphere --spp 1000"
