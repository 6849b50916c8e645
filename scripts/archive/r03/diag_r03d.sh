#!/usr/bin/env bash
# Round 3: strong-scaling shares on one GPU (--part P/N), and the N>1 entry paths on the
# 1-GPU box with the collectives on gloo (ranks share the GPU): self-spawned and torchrun.
# usage: bash scripts/archive/r03/diag_r03d.sh -> gpurun_out/r03d/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r03d"; mkdir -p "$OUT"; cd "$R"
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-12s %9.0f Mray/s  kernel %9.0f  ms/step %.2f  launches/step %s  %s' % (sys.argv[2], d['value'], d['kernel_mrays'] or 0, d['ms_per_step'], d['world']['ranks'][0]['trace_launches'] // d['steps'], d['config']['parallelism']))" "$1" "$2"; }
for p in full 0/2 0/4 0/8 7/8; do
  n=${p//\//_}; args=(); [ "$p" != full ] && args=(--part "$p")
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e "${args[@]}" > "$OUT/part_$n.json" 2> "$OUT/part_$n.log"
  rc=$?; fatal $rc "part $p"; [ $rc -eq 0 ] && show "$OUT/part_$n.json" "part_$n"
done
timeout -k 10 300 env PT_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 2 --warmup 1 --spp 2000 --no-cpu-baseline \
  > "$OUT/spawn2_gloo.json" 2> "$OUT/spawn2_gloo.log"; rc=$?; fatal $rc spawn; echo "spawn rc=$rc"; tail -c 700 "$OUT/spawn2_gloo.json"
timeout -k 10 300 env PT_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --spp 2000 --no-cpu-baseline > "$OUT/torchrun2_gloo.json" 2> "$OUT/torchrun2_gloo.log"
rc=$?; fatal $rc torchrun; echo "torchrun rc=$rc"; tail -c 300 "$OUT/torchrun2_gloo.json"
echo "diag done"
