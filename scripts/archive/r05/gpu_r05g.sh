#!/usr/bin/env bash
# Round 5, box-level pairs: full GPU suite, then A/B of PT_BOX_PAIRS (default on) vs leaf pairs,
# each variant twice, on Cornell, modified Cornell r=0.3 and Cornell depth 8.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
bash scripts/ab.sh \
  "cor_box||--spp 1500" "cor_leaf|PT_BOX_PAIRS=0|--spp 1500" \
  "mc03_box||--scene mcornell --rough 0.3 --spp 1500" "mc03_leaf|PT_BOX_PAIRS=0|--scene mcornell --rough 0.3 --spp 1500" \
  "d8_box||--depth 8 --spp 1000" "d8_leaf|PT_BOX_PAIRS=0|--depth 8 --spp 1000" \
  "cor_box2||--spp 1500" "cor_leaf2|PT_BOX_PAIRS=0|--spp 1500" \
  "mc03_box2||--scene mcornell --rough 0.3 --spp 1500" "mc03_leaf2|PT_BOX_PAIRS=0|--scene mcornell --rough 0.3 --spp 1500" \
  "d8_box2||--depth 8 --spp 1000" "d8_leaf2|PT_BOX_PAIRS=0|--depth 8 --spp 1000"
