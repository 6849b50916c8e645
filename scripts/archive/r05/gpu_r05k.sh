#!/usr/bin/env bash
# Round 5: whole-job A/B of the sparse slab (now off by default; PT_SPARSE=1 on) and of the
# fused accumulation's tail batch (PT_TAIL_DIV 4 / 8), Cornell and config 4, after the GPU suite.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R"
C="--spp 10000"; S="--scene sphere --spp 1000"
bash scripts/ab.sh \
  "cor_def||$C" "cor_sparse|PT_SPARSE=1|$C" "cor_t4|PT_TAIL_DIV=4|$C" "cor_t8|PT_TAIL_DIV=8|$C" \
  "c4_def||$S" "c4_sparse|PT_SPARSE=1|$S" "c4_t4|PT_TAIL_DIV=4|$S" \
  "cor_def2||$C" "cor_sparse2|PT_SPARSE=1|$C" "cor_t42|PT_TAIL_DIV=4|$C" "cor_t82|PT_TAIL_DIV=8|$C" \
  "c4_def2||$S" "c4_sparse2|PT_SPARSE=1|$S" "c4_t42|PT_TAIL_DIV=4|$S"
