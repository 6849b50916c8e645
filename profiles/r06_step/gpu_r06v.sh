#!/usr/bin/env bash
# Round 6: config 5's full frame through the in-process RCCL gather (send-to-self, test hooks on,
# as round 5 measured it), then the headline step's trace outside the kernels (gpu_r06u.sh).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06bal
PT_TEST_HOOKS=1 timeout -k 10 300 python -u scripts/part_balance.py --band 1 --scene cornell --res 4096 --spp 10000 --depth 8 --ns 8 --rccl > gpurun_out/r06bal/cfg5_rccl.json 2> gpurun_out/r06bal/cfg5_rccl.log || { tail -5 gpurun_out/r06bal/cfg5_rccl.log; exit 1; }
tail -2 gpurun_out/r06bal/cfg5_rccl.log
bash scripts/gpu_r06u.sh
