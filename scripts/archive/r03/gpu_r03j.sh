# compact wide triangle records A/B + the GPU suite
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03j/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03j/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
STEPS=3 bash scripts/archive/r03/ab_r03.sh compact "s_c0|PT_WIDE_COMPACT=0|--scene sphere --spp 1000" "s_c1||--scene sphere --spp 1000" \
  "s_c0b|PT_WIDE_COMPACT=0|--scene sphere --spp 1000" "s_c1b||--scene sphere --spp 1000" "c||"
