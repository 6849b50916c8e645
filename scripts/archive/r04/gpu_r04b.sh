#!/usr/bin/env bash
# Round 4: config 4 A/B — one-word queue entries (default lib), more LDS top nodes, and
# batched camera rays (PT_WIDE_PREFETCH=1 variant, its wide-tree parity first).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
V=pathtracer-cpp_amd/lib/variants
PT_LIB=$V/libpt_hip_pf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "wide or multi_batch" > gpurun_out/r04b_pytest_pf.log 2>&1; rc=$?
echo "pytest pf rc=$rc"; tail -3 gpurun_out/r04b_pytest_pf.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "r3:PT_LIB=$V/libpt_hip_r3.so:--scene sphere --spp 1000" \
  "q32::--scene sphere --spp 1000" \
  "q32top8k:PT_WIDE_TOP_BYTES=8192:--scene sphere --spp 1000" \
  "pf:PT_LIB=$V/libpt_hip_pf.so:--scene sphere --spp 1000" \
  "pf_rt16:PT_LIB=$V/libpt_hip_pf.so,PT_REGEN_THRESH=16:--scene sphere --spp 1000" \
  "pf_rt24:PT_LIB=$V/libpt_hip_pf.so,PT_REGEN_THRESH=24:--scene sphere --spp 1000" \
  "pf_rt40:PT_LIB=$V/libpt_hip_pf.so,PT_REGEN_THRESH=40:--scene sphere --spp 1000" \
  "pf_th32:PT_LIB=$V/libpt_hip_pf.so,PT_WIDE_THRESH=32:--scene sphere --spp 1000" \
  "r3b:PT_LIB=$V/libpt_hip_r3.so:--scene sphere --spp 1000" \
  "q32b::--scene sphere --spp 1000"
