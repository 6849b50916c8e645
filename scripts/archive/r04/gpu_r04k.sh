#!/usr/bin/env bash
# Round 4: the scene kernel at 8 waves with the AMDGPU pressure trackers as the default —
# the whole GPU suite, then A/B against 7 waves (PT_RTC_WAVES=7, same flags) on configs
# 2, 3 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r04k/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r04k/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "cor_w7:PT_RTC_WAVES=7:--spp 1000" "cor_w8::--spp 1000" "mc_w7:PT_RTC_WAVES=7:--scene mcornell --rough 0.3 --spp 1000" \
  "mc_w8::--scene mcornell --rough 0.3 --spp 1000" "c5_w7:PT_RTC_WAVES=7:--res 4096 --depth 8 --spp 64" \
  "c5_w8::--res 4096 --depth 8 --spp 64" "cor_w7b:PT_RTC_WAVES=7:--spp 1000" "cor_w8b::--spp 1000"
