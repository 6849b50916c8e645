#!/usr/bin/env bash
# rocprofv3 evidence for the trace kernel (run on the GPU box via gpurun):
#   1. kernel trace + stats of the bench command (per-kernel average durations)
#   2. separate --pmc passes (never combined with other trace domains):
#      FETCH_SIZE, WRITE_SIZE (HBM bytes; gfx950: FETCH_SIZE reads half of a wide
#      coalesced stream, see MI355X_MICROARCH.md §HBM), and SQ instruction counters.
# Usage: bash scripts/profile.sh [TAG] [bench args...]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
shift || true
ARGS=("$@")
if [ ${#ARGS[@]} -eq 0 ]; then ARGS=(--steps 1 --warmup 0 --no-cpu-baseline); fi
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp

run() {  # name, then rocprofv3 options
    local name="$1"; shift
    echo "[profile] $name" >&2
    timeout -k 10 600 rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
        python3 "$R/bench.py" "${ARGS[@]}" > "$OUT/$name.bench.json" 2> "$OUT/$name.log"
    local rc=$?
    echo "[profile] $name rc=$rc" >&2
    return $rc
}

rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
run kt --kernel-trace --stats || exit $?
run pmc_fetch --pmc FETCH_SIZE || exit $?
run pmc_write --pmc WRITE_SIZE || exit $?
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY || exit $?
echo "[profile] done" >&2
