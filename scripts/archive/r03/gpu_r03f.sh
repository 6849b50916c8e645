set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03f
PT_WIDE_F16=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wide or full_size" > gpurun_out/r03f/pytest_f16.log 2>&1; rc=$?
tail -3 gpurun_out/r03f/pytest_f16.log
[ $rc -eq 0 ] || exit $rc
bash scripts/archive/r03/ab_r03.sh f16 "base||--scene sphere --spp 1000" "f16|PT_WIDE_F16=1|--scene sphere --spp 1000" "base2||--scene sphere --spp 1000" "f16b|PT_WIDE_F16=1|--scene sphere --spp 1000"
