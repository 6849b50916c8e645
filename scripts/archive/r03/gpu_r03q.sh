# slab store base / plane and the exact walk's stack from the kernarg segment (A/B vs HEAD)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03q/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03q/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
H=pathtracer-cpp_amd/lib/variants/libpt_hip_head.so
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh store "s_head|PT_LIB=$H|$S" "s_new||$S" "c_head|PT_LIB=$H|" "c_new||" "s_head2|PT_LIB=$H|$S" "s_new2||$S" "c_head2|PT_LIB=$H|" "c_new2||"
