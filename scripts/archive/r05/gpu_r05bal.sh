#!/usr/bin/env bash
# Round 5, final kernel (flagged slabs): every rank's share of configs 2, 4, 5 at N = 2/4/8 with the
# default 1-row bands, timed alone on one GPU (scripts/part_balance.py); config 5's whole
# frame through the in-process RCCL gather (send-to-self).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
mkdir -p gpurun_out/r05bal
export PT_TEST_HOOKS=1
run() {
  local name="$1"; shift
  timeout -k 10 500 python -u scripts/part_balance.py --band 1 "$@" > gpurun_out/r05bal/$name.json 2> gpurun_out/r05bal/$name.log
  local rc=$?; echo "== $name rc=$rc"; tail -4 gpurun_out/r05bal/$name.log; return $rc
}
run cfg2 --scene cornell --res 1024 --spp 10000 --depth 5 --ns 2 4 8 && \
run cfg4 --scene sphere --res 1024 --spp 1000 --depth 5 --ns 2 4 8 --reps 2 && \
run cfg5 --scene cornell --res 4096 --spp 10000 --depth 8 --ns 2 4 8 --rccl
