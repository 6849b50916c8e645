#!/usr/bin/env bash
# Round 5: flagged slabs' separate pass with parallel record loads: one rank's share at N = 8
# and 4 (single- and multi-batch frames) and the headline, against dense slabs (PT_FLAGS=0).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R"
SKIP_TESTS=1 bash scripts/ab.sh \
  "p8_fl||--part 0/8" "p8_dn|PT_FLAGS=0|--part 0/8" "p4_fl||--part 0/4" "p4_dn|PT_FLAGS=0|--part 0/4" \
  "c4p8_fl||--scene sphere --spp 1000 --part 0/8" "c4p8_dn|PT_FLAGS=0|--scene sphere --spp 1000 --part 0/8" \
  "cor_fl||" "cor_dn|PT_FLAGS=0|" \
  "p8_fl2||--part 0/8" "p8_dn2|PT_FLAGS=0|--part 0/8" "p4_fl2||--part 0/4" "p4_dn2|PT_FLAGS=0|--part 0/4"
