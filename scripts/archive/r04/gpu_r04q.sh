#!/usr/bin/env bash
# Round 4: the scene kernel's compile-time switches re-checked at 8 waves (hipRTC defines,
# no rebuild): packed plane pairs, multi-leaf OR, shared clamp off, carry-chain mask off,
# per-level unwinding loop, camera fields from argument registers.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D=PT_RTC_DEFINES
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "cor::--spp 1000" "cor_pk:$D=PT_PK_PLANES=1:--spp 1000" "cor_mlo:$D=PT_MULTI_LEAF_OR=1:--spp 1000" \
  "cor_noclamp:$D=PT_SHARED_CLAMP=0:--spp 1000" "cor_noaddc:$D=PT_ADDC_MASK=0:--spp 1000" \
  "cor_foldloop:$D=PT_FOLD_UNROLL=0:--spp 1000" "cor_camreg:$D=PT_CAM_KERNARG=0:--spp 1000" "cor2::--spp 1000" \
  "mc::--scene mcornell --rough 0.3 --spp 1000" "mc_pk:$D=PT_PK_PLANES=1:--scene mcornell --rough 0.3 --spp 1000" \
  "mc_mlo:$D=PT_MULTI_LEAF_OR=1:--scene mcornell --rough 0.3 --spp 1000" "mc2::--scene mcornell --rough 0.3 --spp 1000"
