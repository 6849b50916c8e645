#!/usr/bin/env bash
# Round 4: radiance slab as [sample][pixel][rgb] (PT_SLAB_RGB=1 variant: one 12-B store per
# finished path) — parity, then A/B on configs 2, 3 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04g
V=$PWD/pathtracer-cpp_amd/lib/variants
T="PT_LIB=$V/libpt_hip_rgb.so,PT_RTC_DEFINES=PT_SLAB_RGB=1"
PT_LIB=$V/libpt_hip_rgb.so PT_RTC_DEFINES=PT_SLAB_RGB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "multi_batch or partition or full_size or wide_tree or vs_oracle" \
  > gpurun_out/r04g/pytest.log 2>&1; rc=$?
echo "pytest rgb rc=$rc"; tail -3 gpurun_out/r04g/pytest.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "cor::--spp 1000" "cor_rgb:$T:--spp 1000" "sph::--scene sphere --spp 1000" "sph_rgb:$T:--scene sphere --spp 1000" \
  "mc::--scene mcornell --rough 0.3 --spp 1000" "mc_rgb:$T:--scene mcornell --rough 0.3 --spp 1000" \
  "cor2::--spp 1000" "cor_rgb2:$T:--spp 1000" "sph2::--scene sphere --spp 1000" "sph_rgb2:$T:--scene sphere --spp 1000"
