# wide step: offsets by base select, mask-only zeroing; LDS top levels on/off (A/B vs HEAD)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03m
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wide or full_size or obj" > gpurun_out/r03m/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03m/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
H=pathtracer-cpp_amd/lib/variants/libpt_hip_head.so
N=pathtracer-cpp_amd/lib/variants/libpt_hip_notop.so
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh step "s_head|PT_LIB=$H|$S" "s_new||$S" "s_notop|PT_LIB=$N|$S" \
  "s_head2|PT_LIB=$H|$S" "s_new2||$S" "s_notop2|PT_LIB=$N|$S"
