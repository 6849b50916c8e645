#!/usr/bin/env bash
# Round 6: the headline frame's last batch (summed by pt_accumulate_kernel after the last launch:
# 2.07 ms over 1812 spp) made small (PT_TAIL_DIV: the last batch = batch / div) — whole job x2.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
SKIP_TESTS=1 bash scripts/ab.sh "td0||--steps 3 --no-e2e" "td8|PT_TAIL_DIV=8|--steps 3 --no-e2e" "td16|PT_TAIL_DIV=16|--steps 3 --no-e2e" \
  "td0b||--steps 3 --no-e2e" "td8b|PT_TAIL_DIV=8|--steps 3 --no-e2e" "td16b|PT_TAIL_DIV=16|--steps 3 --no-e2e" \
  "c5td0||--res 4096 --depth 8 --steps 1 --no-e2e" "c5td8|PT_TAIL_DIV=8|--res 4096 --depth 8 --steps 1 --no-e2e"
