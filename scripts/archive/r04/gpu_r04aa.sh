#!/usr/bin/env bash
# Round 4, final kernel: camera-ray regeneration threshold re-checked (runtime hook).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "c32::--spp 1000" "c40:PT_REGEN_THRESH=40:--spp 1000" "c24:PT_REGEN_THRESH=24:--spp 1000" \
  "c32b::--spp 1000" "c40b:PT_REGEN_THRESH=40:--spp 1000" "c28:PT_REGEN_THRESH=28:--spp 1000" "c36:PT_REGEN_THRESH=36:--spp 1000" \
  "m32::--scene mcornell --rough 0.3 --spp 1000" "m40:PT_REGEN_THRESH=40:--scene mcornell --rough 0.3 --spp 1000" \
  "m32b::--scene mcornell --rough 0.3 --spp 1000" "m40b:PT_REGEN_THRESH=40:--scene mcornell --rough 0.3 --spp 1000"
