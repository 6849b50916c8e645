# flat kernel: path-record bases and the fold's unroll test from the kernarg segment (A/B vs HEAD)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03p
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03p/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03p/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
H=pathtracer-cpp_amd/lib/variants/libpt_hip_head.so
M="--scene mcornell --rough 0.3"
STEPS=3 bash scripts/archive/r03/ab_r03.sh recs "c_head|PT_LIB=$H|" "c_new||" "mc_head|PT_LIB=$H|$M" "mc_new||$M" "c_head2|PT_LIB=$H|" "c_new2||" \
  "c8_head|PT_LIB=$H|--res 4096 --depth 8 --spp 1000" "c8_new||--res 4096 --depth 8 --spp 1000"
