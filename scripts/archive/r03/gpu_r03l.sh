# 32-bit work pool + countdown cadence A/B against HEAD's library, and the flat kernel at 8 waves
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03l/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03l/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
H=pathtracer-cpp_amd/lib/variants/libpt_hip_head.so
STEPS=3 bash scripts/archive/r03/ab_r03.sh pool \
  "c_head|PT_LIB=$H|" "c_new||" "c_new8|PT_RTC_WAVES=8|" \
  "mc_head|PT_LIB=$H|--scene mcornell --rough 0.3" "mc_new||--scene mcornell --rough 0.3" "mc_new8|PT_RTC_WAVES=8|--scene mcornell --rough 0.3" \
  "s_head|PT_LIB=$H|--scene sphere --spp 1000" "s_new||--scene sphere --spp 1000" \
  "c_head2|PT_LIB=$H|" "c_new2||" "c_new82|PT_RTC_WAVES=8|"
