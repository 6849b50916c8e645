#!/usr/bin/env bash
# Round 4: one margin per ray segment in the wide walk (PT_WIDE_RAY_MARGIN=1 variant):
# parity on the wide kernel, VALU per ray and A/B on config 4; the walk's threshold again.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04f
V=$PWD/pathtracer-cpp_amd/lib/variants
PT_LIB=$V/libpt_hip_rmargin.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "wide or full_size or multi_batch" \
  > gpurun_out/r04f/pytest.log 2>&1; rc=$?
echo "pytest rmargin rc=$rc"; tail -3 gpurun_out/r04f/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_valu.sh rm 'base||--scene sphere --spp 250' "rm|PT_LIB=$V/libpt_hip_rmargin.so|--scene sphere --spp 250" || exit $?
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "sph::--scene sphere --spp 1000" "sph_rm:PT_LIB=$V/libpt_hip_rmargin.so:--scene sphere --spp 1000" \
  "sph_th24:PT_WIDE_THRESH=24:--scene sphere --spp 1000" "sph_th32:PT_WIDE_THRESH=32:--scene sphere --spp 1000" \
  "sph_rm_th32:PT_LIB=$V/libpt_hip_rmargin.so,PT_WIDE_THRESH=32:--scene sphere --spp 1000" \
  "sph2::--scene sphere --spp 1000" "sph_rm2:PT_LIB=$V/libpt_hip_rmargin.so:--scene sphere --spp 1000"
