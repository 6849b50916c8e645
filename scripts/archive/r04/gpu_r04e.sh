#!/usr/bin/env bash
# Round 4: adaptive theta table (PT_THETA_TAB=2 variant: waves with few sampling lanes read
# the table) — parity, then A/B on configs 2, 3, 4; and the row partition with 1-row bands.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04e
V=$PWD/pathtracer-cpp_amd/lib/variants
T="PT_LIB=$V/libpt_hip_theta2.so,PT_RTC_DEFINES=PT_THETA_TAB=2"
PT_LIB=$V/libpt_hip_theta2.so PT_RTC_DEFINES=PT_THETA_TAB=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "vs_oracle or golden_images or wide_tree_bitexact or full_size" \
  > gpurun_out/r04e/pytest.log 2>&1; rc=$?
echo "pytest theta2 rc=$rc"; tail -3 gpurun_out/r04e/pytest.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "cor::--spp 1000" "cor_t16:$T:--spp 1000" "cor_t32:$T,PT_THETA_LANES=32:--spp 1000" \
  "mc::--scene mcornell --rough 0.3 --spp 1000" "mc_t16:$T:--scene mcornell --rough 0.3 --spp 1000" \
  "mc_t32:$T,PT_THETA_LANES=32:--scene mcornell --rough 0.3 --spp 1000" \
  "mc_t64:$T,PT_THETA_LANES=64:--scene mcornell --rough 0.3 --spp 1000" \
  "sph::--scene sphere --spp 1000" "sph_t16:$T:--scene sphere --spp 1000" "sph_t8:$T,PT_THETA_LANES=8:--scene sphere --spp 1000" || exit $?
export PT_TEST_HOOKS=1
timeout -k 10 300 python -u scripts/part_balance.py --scene sphere --res 1024 --spp 1000 --depth 5 --ns 8 --reps 2 --band 1 \
  > gpurun_out/r04e/cfg4_band1.json 2> gpurun_out/r04e/cfg4_band1.log && tail -2 gpurun_out/r04e/cfg4_band1.log && \
timeout -k 10 300 python -u scripts/part_balance.py --scene cornell --res 1024 --spp 10000 --depth 5 --ns 8 --band 1 \
  > gpurun_out/r04e/cfg2_band1.json 2> gpurun_out/r04e/cfg2_band1.log && tail -2 gpurun_out/r04e/cfg2_band1.log
