#!/usr/bin/env bash
# Round 4: multi-GPU balance evidence on one GPU. Every rank's share of the
# row partition at N = 2/4/8 timed alone for config 5 (Cornell 4096², 10k spp, depth 8),
# config 4 (99k mesh) and the headline; config 5's full frame once through the in-process
# RCCL gather (send-to-self) for its gather time.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04c
export PT_TEST_HOOKS=1
run() {  # name, args
  local name="$1"; shift
  timeout -k 10 500 python -u scripts/part_balance.py "$@" > gpurun_out/r04c/$name.json 2> gpurun_out/r04c/$name.log
  local rc=$?
  echo "== $name rc=$rc"; tail -4 gpurun_out/r04c/$name.log
  return $rc
}
run cfg5 --scene cornell --res 4096 --spp 10000 --depth 8 --ns 2 4 8 --rccl && \
run cfg4 --scene sphere --res 1024 --spp 1000 --depth 5 --ns 2 4 8 --reps 2 && \
run cfg2 --scene cornell --res 1024 --spp 10000 --depth 5 --ns 2 4 8
