#!/usr/bin/env bash
# Round 6: float child planes in the wide walk (PT_WIDE_PLANES=f32) — parity, then config 4 A/B.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06a
W5="$R/pathtracer-cpp_amd/lib/variants/libpt_hip_w5.so"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "wide_tree_bitexact or dark_path_skip" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06a/pytest_wide.log 2>&1
rc=$?; echo "pytest wide rc=$rc"; tail -3 gpurun_out/r06a/pytest_wide.log; [ $rc -eq 0 ] || exit $rc
PT_WIDE_PLANES=f32 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "random_scenes or full_size or wide_walk_exact" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06a/pytest_f32.log 2>&1
rc=$?; echo "pytest f32 rc=$rc"; tail -3 gpurun_out/r06a/pytest_f32.log; [ $rc -eq 0 ] || exit $rc
S="--scene sphere --spp 1000 --no-e2e"
SKIP_TESTS=1 bash scripts/ab.sh "c4_f16||$S" "c4_f32|PT_WIDE_PLANES=f32|$S" "c4_f32w5|PT_WIDE_PLANES=f32 PT_LIB=$W5|$S" \
  "c4_f16w5|PT_LIB=$W5|$S" "c4_f32w4w5|PT_WIDE_PLANES=f32 PT_WIDE_W=4 PT_LIB=$W5|$S" "c4_f32w4|PT_WIDE_PLANES=f32 PT_WIDE_W=4|$S" \
  "c4_f16b||$S" "c4_f32b|PT_WIDE_PLANES=f32|$S" "c4_f32w5b|PT_WIDE_PLANES=f32 PT_LIB=$W5|$S"
