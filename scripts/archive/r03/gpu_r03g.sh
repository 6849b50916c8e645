set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wide or full_size or obj" > gpurun_out/r03g/pytest_sah.log 2>&1; rc=$?
tail -3 gpurun_out/r03g/pytest_sah.log
[ $rc -eq 0 ] || exit $rc
bash scripts/archive/r03/ab_r03.sh sah "greedy|PT_WIDE_COLLAPSE=greedy|--scene sphere --spp 1000" "sah||--scene sphere --spp 1000" "greedy2|PT_WIDE_COLLAPSE=greedy|--scene sphere --spp 1000" "sah2||--scene sphere --spp 1000"
