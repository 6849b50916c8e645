#!/usr/bin/env bash
# Round 4, final kernel: timing bounds of the flat kernel's sections at 8 waves (wrong
# images; hipRTC defines): no unwinding, no hemisphere sample, no radiance stores, no
# triangle tests (first passing leaf), no fused accumulation.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D=PT_RTC_DEFINES
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "cor::--spp 1000" "nofold:$D=PT_EXP_NO_FOLD=1:--spp 1000" "nobrdf:$D=PT_EXP_NO_BRDF=1:--spp 1000" \
  "nostore:$D=PT_EXP_NO_STORE=1:--spp 1000" "nopairs:$D=PT_EXP_NO_PAIRS=1:--spp 1000" "cor2::--spp 1000" \
  "nofold2:$D=PT_EXP_NO_FOLD=1:--spp 1000"
