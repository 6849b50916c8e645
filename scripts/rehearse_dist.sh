#!/usr/bin/env bash
# Rehearsal of bench.py's N>1 path on a box with fewer GPUs than ranks: torchrun with N
# ranks, the collectives on gloo and rank r on GPU r mod count (PT_BENCH_BACKEND=gloo).
# Checks the partition, the frame gather to rank 0 and the max-over-ranks timing; the
# RCCL leg itself needs one GPU per rank (the driver's multi-GPU run).
# usage: bash scripts/rehearse_dist.sh "2 4" [bench args]   -> gpurun_out/reh/n<N>.json
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
NS="$1"; shift
cd "$R" && mkdir -p gpurun_out/reh
port=29511
for n in $NS; do
  PT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus "$n" "$@" \
    > gpurun_out/reh/n$n.json 2> gpurun_out/reh/n$n.log || { echo "n=$n failed"; tail -5 gpurun_out/reh/n$n.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('n=%s %.0f Mray/s  %s' % (sys.argv[2], d['value'], d['config']['parallelism']))" gpurun_out/reh/n$n.json $n
  port=$((port + 1))
done
