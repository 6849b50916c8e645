# wide kernel: camera rays prefetched in LDS (flat kernel's scheme), walk stack rows 9 in LDS + HBM overflow
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03v
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03v/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03v/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
H=pathtracer-cpp_amd/lib/variants/libpt_hip_head.so
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh pref "s_head|PT_LIB=$H|$S" "s_new||$S" "s_r7|PT_WIDE_LDS_ROWS=7|$S" "s_t16|PT_REGEN_THRESH=16|$S" "s_t48|PT_REGEN_THRESH=48|$S" \
  "s_head2|PT_LIB=$H|$S" "s_new2||$S" "c_head|PT_LIB=$H|" "c_new||"
