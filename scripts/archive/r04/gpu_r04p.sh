#!/usr/bin/env bash
# Round 4: keyed PMC evidence of the final kernel sources (all ten config workloads), then
# where a process's first context creation spends its time (scripts/ctx_timing.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash scripts/evidence_all.sh r04 || exit $?
timeout -k 10 200 python scripts/ctx_timing.py > gpurun_out/ctx_timing.txt 2>&1; cat gpurun_out/ctx_timing.txt
