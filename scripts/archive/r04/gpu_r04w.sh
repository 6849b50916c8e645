#!/usr/bin/env bash
# Round 4: radiance-slab budget per launch (PT_BATCH_BYTES; default 16 GiB = 1365 spp of a
# 1024^2 frame per launch) at 32 / 64 GiB: fewer launches per 10k-spp frame, fewer drain
# tails. Full headline frames (whole job, 2 steps each).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04w
for spec in "b16:" "b32:PT_BATCH_BYTES=34359738368" "b64:PT_BATCH_BYTES=68719476736" "b16b:" "b32b:PT_BATCH_BYTES=34359738368"; do
  n=${spec%%:*}; e=${spec#*:}
  timeout -k 10 300 env PT_TEST_HOOKS=1 $e python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e \
    > gpurun_out/r04w/$n.json 2> gpurun_out/r04w/$n.log || { echo "$n failed"; tail -3 gpurun_out/r04w/$n.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r04w/$n.json')); print('$n', 'Mray/s=%.0f'%d['value'], 'ms/step=%.1f'%d['ms_per_step'], 'launches', d.get('roofline',{}).get('avg_launch_ms'))"
done
