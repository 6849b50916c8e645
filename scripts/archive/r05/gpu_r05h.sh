#!/usr/bin/env bash
# Round 5: where the cold start's context creation goes (scripts/ctx_timing.py), two processes.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/ctx
for i in 1 2; do
  timeout -k 10 180 python -u scripts/ctx_timing.py > gpurun_out/ctx/t$i.json 2> gpurun_out/ctx/t$i.log || exit $?
  cat gpurun_out/ctx/t$i.json; grep pt_ctx_create gpurun_out/ctx/t$i.log
done
