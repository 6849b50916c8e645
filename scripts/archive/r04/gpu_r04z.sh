#!/usr/bin/env bash
# Round 4: the scene kernel without fresh_tid() re-reads (PT_FRESH_TID=0: 55 VGPRs, no
# scratch at 8 waves now that the camera terms sit in SGPRs) against the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
F=PT_RTC_DEFINES=PT_FRESH_TID=0
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "c1::--spp 1000" "c1_ft0:$F:--spp 1000" "c2::--spp 1000" "c2_ft0:$F:--spp 1000" "c3::--spp 1000" "c3_ft0:$F:--spp 1000" \
  "m1::--scene mcornell --rough 0.3 --spp 1000" "m1_ft0:$F:--scene mcornell --rough 0.3 --spp 1000" \
  "m2::--scene mcornell --rough 0.3 --spp 1000" "m2_ft0:$F:--scene mcornell --rough 0.3 --spp 1000" \
  "s1::--res 4096 --depth 8 --spp 64" "s1_ft0:$F:--res 4096 --depth 8 --spp 64"
