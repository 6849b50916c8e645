# wide kernel: one-byte material-row records (LDS), and 7 waves per SIMD with a shorter queue
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03r
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wide or full_size or obj" > gpurun_out/r03r/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03r/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
H=pathtracer-cpp_amd/lib/variants/libpt_hip_head.so
W7=pathtracer-cpp_amd/lib/variants/libpt_hip_w7.so
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh w7 "s_head|PT_LIB=$H|$S" "s_new||$S" "s_new_q112|PT_WIDE_QUEUE_LEN=112|$S" \
  "s_w7_q112|PT_LIB=$W7 PT_WIDE_QUEUE_LEN=112|$S" "s_w7_q96|PT_LIB=$W7 PT_WIDE_QUEUE_LEN=96|$S" \
  "s_head2|PT_LIB=$H|$S" "s_new2||$S" "s_w7_q112b|PT_LIB=$W7 PT_WIDE_QUEUE_LEN=112|$S"
