#!/usr/bin/env bash
# Round 5: flagged slabs (dark scenes: only non-dark paths store, the accumulation reads the
# bits and only flagged records) against dense slabs (PT_FLAGS=0), whole job; after the suite.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R"
bash scripts/ab.sh \
  "cor_fl||" "cor_dn|PT_FLAGS=0|" "mc3_fl||--scene mcornell --rough 0.3 --spp 3000" "mc3_dn|PT_FLAGS=0|--scene mcornell --rough 0.3 --spp 3000" \
  "c4_fl||--scene sphere --spp 1000" "c4_dn|PT_FLAGS=0|--scene sphere --spp 1000" \
  "p8_fl||--part 0/8" "p8_dn|PT_FLAGS=0|--part 0/8" "c5_fl||--res 4096 --depth 8 --spp 300" "c5_dn|PT_FLAGS=0|--res 4096 --depth 8 --spp 300" \
  "cor_fl2||" "cor_dn2|PT_FLAGS=0|" "mc3_fl2||--scene mcornell --rough 0.3 --spp 3000" "mc3_dn2|PT_FLAGS=0|--scene mcornell --rough 0.3 --spp 3000" \
  "c4_fl2||--scene sphere --spp 1000" "c4_dn2|PT_FLAGS=0|--scene sphere --spp 1000" \
  "p8_fl2||--part 0/8" "p8_dn2|PT_FLAGS=0|--part 0/8"
