#!/usr/bin/env bash
# Round 4: unwinding with pre-doubled albedo (kAlbedoX2) — parity, then A/B against
# PT_ALBEDO_X2=0 on configs 2, 3 and 5 (depth 8: the per-level loop).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04i
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "albedo_x2 or vs_oracle or golden_images or multi_batch or full_size" \
  > gpurun_out/r04i/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r04i/pytest.log; [ $rc -eq 0 ] || exit $rc
O=PT_ALBEDO_X2=0
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "cor_x1:$O:--spp 1000" "cor_x2::--spp 1000" "mc_x1:$O:--scene mcornell --rough 0.3 --spp 1000" \
  "mc_x2::--scene mcornell --rough 0.3 --spp 1000" "c5_x1:$O:--res 4096 --depth 8 --spp 64" \
  "c5_x2::--res 4096 --depth 8 --spp 64" \
  "cor_x1b:$O:--spp 1000" "cor_x2b::--spp 1000" "mc_x1b:$O:--scene mcornell --rough 0.3 --spp 1000" \
  "mc_x2b::--scene mcornell --rough 0.3 --spp 1000"
