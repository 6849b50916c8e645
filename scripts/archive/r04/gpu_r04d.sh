#!/usr/bin/env bash
# Round 4: hemisphere_sample's theta terms from a device table (PT_THETA_TAB variant):
# parity on the flat (hipRTC) and wide kernels, then A/B on configs 2, 3 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
V=$PWD/pathtracer-cpp_amd/lib/variants
PT_LIB=$V/libpt_hip_theta.so PT_RTC_DEFINES=PT_THETA_TAB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "vs_oracle or golden_images or wide_tree_bitexact or full_size" \
  > gpurun_out/r04d_pytest.log 2>&1; rc=$?
echo "pytest theta rc=$rc"; tail -3 gpurun_out/r04d_pytest.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "cor::--spp 1000" \
  "cor_theta:PT_LIB=$V/libpt_hip_theta.so,PT_RTC_DEFINES=PT_THETA_TAB=1:--spp 1000" \
  "sph::--scene sphere --spp 1000" \
  "sph_theta:PT_LIB=$V/libpt_hip_theta.so:--scene sphere --spp 1000" \
  "mc::--scene mcornell --rough 0.3 --spp 1000" \
  "mc_theta:PT_LIB=$V/libpt_hip_theta.so,PT_RTC_DEFINES=PT_THETA_TAB=1:--scene mcornell --rough 0.3 --spp 1000" \
  "cor2::--spp 1000" \
  "cor_theta2:PT_LIB=$V/libpt_hip_theta.so,PT_RTC_DEFINES=PT_THETA_TAB=1:--spp 1000"
