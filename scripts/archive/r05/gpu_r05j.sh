#!/usr/bin/env bash
# Round 5: the dark-path skip A/B on the configs VERDICT r4 #2 names that round 5's first A/B
# did not cover: modified Cornell r = 0.8 and config 5 (Cornell 4096^2, depth 8; 300 spp for
# the A/B). Default (skip + sparse slab), PT_SPARSE=0 (skip only), PT_DARK=0 (neither).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R"
M="--scene mcornell --rough 0.8 --spp 1500"; F="--res 4096 --depth 8 --spp 300"
SKIP_TESTS=1 bash scripts/ab.sh \
  "mc08_dark||$M" "mc08_nosparse|PT_SPARSE=0|$M" "mc08_full|PT_DARK=0|$M" \
  "c5_dark||$F" "c5_nosparse|PT_SPARSE=0|$F" "c5_full|PT_DARK=0|$F" \
  "mc08_dark2||$M" "mc08_nosparse2|PT_SPARSE=0|$M" "mc08_full2|PT_DARK=0|$M" \
  "c5_dark2||$F" "c5_nosparse2|PT_SPARSE=0|$F" "c5_full2|PT_DARK=0|$F"
