#!/usr/bin/env bash
# Full bench (default args, with CPU baseline) + rocprofv3 evidence for the same command.
# usage: bash scripts/round_evidence.sh TAG
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
OUT="$R/gpurun_out/ev_$TAG"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
PB=(--steps 1 --warmup 0 --no-cpu-baseline)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 "$R/bench.py" "${PB[@]}" > "$OUT/kt.json" 2> "$OUT/kt.log" || { echo "kt failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 "$R/bench.py" "${PB[@]}" > "$OUT/fetch.json" 2> "$OUT/fetch.log" || { echo "fetch failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 "$R/bench.py" "${PB[@]}" > "$OUT/write.json" 2> "$OUT/write.log" || { echo "write failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -d "$OUT/sq" -o sq --output-format csv -- python3 "$R/bench.py" "${PB[@]}" > "$OUT/sq.json" 2> "$OUT/sq.log" || { echo "sq failed"; exit 1; }
cat "$OUT/kt/kt_kernel_stats.csv"
echo done
