# camera fields from the kernarg segment (fewer SGPR spill lanes): A/B on configs 2, 3, 4
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03o/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03o/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
V=pathtracer-cpp_amd/lib/variants/libpt_hip_camsgpr.so
S="--scene sphere --spp 1000"; M="--scene mcornell --rough 0.3"
STEPS=3 bash scripts/archive/r03/ab_r03.sh cam "c_old|PT_RTC_DEFINES=PT_CAM_KERNARG=0|" "c_new||" "mc_old|PT_RTC_DEFINES=PT_CAM_KERNARG=0|$M" "mc_new||$M" \
  "s_old|PT_LIB=$V|$S" "s_new||$S" "c_old2|PT_RTC_DEFINES=PT_CAM_KERNARG=0|" "c_new2||"
