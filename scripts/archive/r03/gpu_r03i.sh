# fresh_tid A/B (no scratch reloads in the megakernel loops) + the GPU suite
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03i
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03i/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03i/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
V=pathtracer-cpp_amd/lib/variants/libpt_hip_nofresh.so
STEPS=3 bash scripts/archive/r03/ab_r03.sh fresh "c_old|PT_RTC_DEFINES=PT_FRESH_TID=0|" "c_new||" "s_old|PT_LIB=$V|--scene sphere --spp 1000" "s_new||--scene sphere --spp 1000" \
  "c_old2|PT_RTC_DEFINES=PT_FRESH_TID=0|" "c_new2||" "s_old2|PT_LIB=$V|--scene sphere --spp 1000" "s_new2||--scene sphere --spp 1000"
