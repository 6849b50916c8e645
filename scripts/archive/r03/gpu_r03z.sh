# wide walk defaults: queue 160, LDS top nodes up to what keeps the occupancy (vs HEAD), + GPU suite
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03z
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03z/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03z/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
H=pathtracer-cpp_amd/lib/variants/libpt_hip_head.so
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh wdef "s_head|PT_LIB=$H|$S" "s_new||$S" "s_head2|PT_LIB=$H|$S" "s_new2||$S" "s_new_d8|PT_LIB=|$S --depth 8" "s_head_d8|PT_LIB=$H|$S --depth 8"
