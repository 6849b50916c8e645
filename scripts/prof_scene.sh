#!/usr/bin/env bash
# rocprofv3 kernel trace + PMC passes of one short bench run (any scene).
# usage: bash scripts/prof_scene.sh TAG "bench args"    -> gpurun_out/prof_TAG/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; ARGS="$2"
OUT="$R/gpurun_out/prof_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B=(python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline $ARGS)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${B[@]}" > "$OUT/kt.json" 2> "$OUT/kt.log" || { echo "kt failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -d "$OUT/sq" -o sq --output-format csv -- "${B[@]}" > "$OUT/sq.json" 2> "$OUT/sq.log" || { echo "sq failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d "$OUT/tcc" -o tcc --output-format csv -- "${B[@]}" > "$OUT/tcc.json" 2> "$OUT/tcc.log" || { echo "tcc failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- "${B[@]}" > "$OUT/fetch.json" 2> "$OUT/fetch.log" || { echo "fetch failed"; exit 1; }
grep -h trace "$OUT/kt/kt_kernel_stats.csv" | head -3
echo "prof $TAG done"
