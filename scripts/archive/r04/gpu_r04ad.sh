#!/usr/bin/env bash
# Round 4, final kernel (pair queues sized for occupancy): config 5's per-rank shares at
# N = 2/4/8 (1-row bands) timed alone, and its whole frame through the RCCL gather.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04ad
export PT_TEST_HOOKS=1
timeout -k 10 500 python -u scripts/part_balance.py --band 1 --scene cornell --res 4096 --spp 10000 --depth 8 --ns 2 4 8 --rccl \
  > gpurun_out/r04ad/cfg5.json 2> gpurun_out/r04ad/cfg5.log; rc=$?; echo "rc=$rc"; tail -3 gpurun_out/r04ad/cfg5.log; exit $rc
