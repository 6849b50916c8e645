#!/usr/bin/env bash
# Round 5: split one-batch frames (the first batch summed inside a second launch) on one
# rank's share at N = 8 and 4 (bench.py --part), against PT_SPLIT_DIV=0; after the GPU suite.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R"
bash scripts/ab.sh \
  "p8||--part 0/8" "p8_off|PT_SPLIT_DIV=0|--part 0/8" "p8_d4|PT_SPLIT_DIV=4|--part 0/8" "p8_d16|PT_SPLIT_DIV=16|--part 0/8" \
  "p4||--part 0/4" "p4_off|PT_SPLIT_DIV=0|--part 0/4" \
  "c4p8||--scene sphere --spp 1000 --part 0/8" "c4p8_off|PT_SPLIT_DIV=0|--scene sphere --spp 1000 --part 0/8" \
  "p8b||--part 0/8" "p8_offb|PT_SPLIT_DIV=0|--part 0/8" "p8_d4b|PT_SPLIT_DIV=4|--part 0/8" "p8_d16b|PT_SPLIT_DIV=16|--part 0/8" \
  "p4b||--part 0/4" "p4_offb|PT_SPLIT_DIV=0|--part 0/4" \
  "c4p8b||--scene sphere --spp 1000 --part 0/8" "c4p8_offb|PT_SPLIT_DIV=0|--scene sphere --spp 1000 --part 0/8"
