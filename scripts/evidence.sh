#!/usr/bin/env bash
# rocprofv3 evidence for one bench workload (run on the GPU box via gpurun):
#   kt      kernel trace + stats (per-kernel average durations)
#   fetch   --pmc FETCH_SIZE            (gfx950: counts half of a wide streaming read, x2)
#   write   --pmc WRITE_SIZE
#   sq      --pmc SQ instruction / wait / lane-utilisation counters
#   tcc     --pmc TCC_HIT_sum TCC_MISS_sum
#   sq2     --pmc SQ_ACTIVE_INST_VALU2 (+ VALU, ANY, GRBM_GUI_ACTIVE): the VALU main-port slots
#           the roofline divides (second-port issue is subtracted)
# Each PMC group is its own run (never combined with other trace domains). Every run is
# one timed step without warm-up, CPU baseline or end-to-end pass, so the trace kernel's
# dispatches are exactly one frame's launches. FULL=1 first runs the complete bench line
# (CPU baseline + end to end) into bench.json.
# usage: bash scripts/evidence.sh TAG [bench args...]   -> gpurun_out/ev_TAG/
#        then (here): python scripts/summarize_profile.py TAG
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
ARGS=("$@")
OUT="$R/gpurun_out/ev_$TAG"
mkdir -p "$OUT"
if [ -n "${FULL:-}" ]; then
  (cd "$R" && timeout -k 10 900 python3 bench.py "${ARGS[@]}" > "$OUT/bench.json" 2> "$OUT/bench.log") \
    || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
  tail -c 600 "$OUT/bench.json"
fi
cd /tmp && export TMPDIR=/tmp
B=(python3 "$R/bench.py" "${ARGS[@]}" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${B[@]}" \
  > "$OUT/kt.json" 2> "$OUT/kt.log" || { echo "kt failed"; tail -5 "$OUT/kt.log"; exit 1; }
for spec in "fetch:FETCH_SIZE" "write:WRITE_SIZE" \
            "sq:SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
            "tcc:TCC_HIT_sum TCC_MISS_sum" \
            "sq2:SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE"; do
  name="${spec%%:*}"; read -r -a CS <<< "${spec#*:}"
  timeout -s KILL 300 rocprofv3 --pmc "${CS[@]}" -d "$OUT/$name" -o "$name" --output-format csv -- "${B[@]}" \
    > "$OUT/$name.json" 2> "$OUT/$name.log" || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
done
grep -h "trace" "$OUT/kt/kt_kernel_stats.csv" | head -3
echo "evidence $TAG done"
