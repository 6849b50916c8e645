# wide step: LDS top levels addressed from LDS address 0, run constants in the load offsets (A/B vs HEAD)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03n
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wide or full_size or obj" > gpurun_out/r03n/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03n/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
H=pathtracer-cpp_amd/lib/variants/libpt_hip_head.so
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh lds0 "s_head|PT_LIB=$H|$S" "s_new||$S" "s_head2|PT_LIB=$H|$S" "s_new2||$S"
