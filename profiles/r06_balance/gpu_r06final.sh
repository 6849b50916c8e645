#!/usr/bin/env bash
# Round 6, final build: one bench line per config (scripts/configs.sh r06, each with its CPU
# baseline and end-to-end pass), then every rank's share of configs 2, 4, 5 at N = 2/4/8
# (scripts/part_balance.py, 1-row bands) and config 5's frame through the RCCL gather.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06bal
bash scripts/configs.sh r06 || exit 1
run() {
  local name="$1"; shift
  timeout -k 10 500 python -u scripts/part_balance.py --band 1 "$@" > gpurun_out/r06bal/$name.json 2> gpurun_out/r06bal/$name.log
  local rc=$?; echo "== $name rc=$rc"; tail -4 gpurun_out/r06bal/$name.log; return $rc
}
run cfg2 --scene cornell --res 1024 --spp 10000 --depth 5 --ns 2 4 8 && \
run cfg4 --scene sphere --res 1024 --spp 1000 --depth 5 --ns 2 4 8 --reps 2 && \
run cfg5 --scene cornell --res 4096 --spp 10000 --depth 8 --ns 2 4 8 --rccl
