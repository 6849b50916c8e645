#!/usr/bin/env bash
# Round 4: cost of the specular rejection loop (config 3) by duplication (PT_EXP_DUP_SPEC,
# hipRTC define), one keyed-free PMC pass each; r = 0 / 0.3 / 0.8.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D=PT_RTC_DEFINES=PT_EXP_DUP_SPEC=1
bash scripts/pmc_valu.sh spec \
  "mc0||--scene mcornell --rough 0 --spp 1000" \
  "mc0_dup|$D|--scene mcornell --rough 0 --spp 1000" \
  "mc03||--scene mcornell --rough 0.3 --spp 1000" \
  "mc03_dup|$D|--scene mcornell --rough 0.3 --spp 1000" \
  "mc08||--scene mcornell --rough 0.8 --spp 1000" \
  "mc08_dup|$D|--scene mcornell --rough 0.8 --spp 1000"
# upper bound of moving the unwinding out of the trace kernel: no fold at all (wrong images)
SKIP_TESTS=1 bash scripts/gpu_ab.sh "cor::--spp 1000" "cor_nofold:PT_RTC_DEFINES=PT_EXP_NO_FOLD=1:--spp 1000" \
  "cor2::--spp 1000" "cor_nofold2:PT_RTC_DEFINES=PT_EXP_NO_FOLD=1:--spp 1000" \
  "mc08::--scene mcornell --rough 0.8 --spp 1000" "mc08_dup:$D:--scene mcornell --rough 0.8 --spp 1000"
