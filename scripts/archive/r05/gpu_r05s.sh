#!/usr/bin/env bash
# Round 5, flagged slabs: the theta table's per-wave threshold re-swept (PT_THETA_LANES; default
# 32 in specular scenes, 0 otherwise) on config 3 r = 0.3 / 0.8, Cornell and config 4.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R"
M="--scene mcornell --rough 0.3 --spp 3000"; M8="--scene mcornell --rough 0.8 --spp 3000"
SKIP_TESTS=1 bash scripts/ab.sh \
  "m3_32||$M" "m3_16|PT_THETA_LANES=16|$M" "m3_48|PT_THETA_LANES=48|$M" \
  "m8_32||$M8" "m8_48|PT_THETA_LANES=48|$M8" \
  "cor_0||--spp 3000" "cor_8|PT_THETA_LANES=8|--spp 3000" "cor_16|PT_THETA_LANES=16|--spp 3000" \
  "c4_0||--scene sphere --spp 1000" "c4_16|PT_THETA_LANES=16|--scene sphere --spp 1000" \
  "m3_32b||$M" "m3_16b|PT_THETA_LANES=16|$M" "m3_48b|PT_THETA_LANES=48|$M" \
  "cor_0b||--spp 3000" "cor_8b|PT_THETA_LANES=8|--spp 3000" "cor_16b|PT_THETA_LANES=16|--spp 3000"
