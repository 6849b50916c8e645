#!/usr/bin/env bash
# Round 5: the sparse slab on config 3 (modified Cornell r = 0 and 0.3), whole job, one box.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R"
A="--scene mcornell --rough 0 --spp 3000"; B="--scene mcornell --rough 0.3 --spp 3000"
SKIP_TESTS=1 bash scripts/ab.sh \
  "m0_def||$A" "m0_sp|PT_SPARSE=1|$A" "m3_def||$B" "m3_sp|PT_SPARSE=1|$B" \
  "m0_def2||$A" "m0_sp2|PT_SPARSE=1|$A" "m3_def2||$B" "m3_sp2|PT_SPARSE=1|$B"
