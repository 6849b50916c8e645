#!/usr/bin/env bash
# Round 5 end, part A: the round-end rehearsal (whole GPU suite, smoke(), default bench line)
# into gpurun_out/final_r05, then keyed PMC evidence for Cornell (with the full bench line),
# config 4, config 1 and modified Cornell r = 0.3 (scripts/evidence.sh).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/final_r05
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/final_r05/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/final_r05/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_r05/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/final_r05/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/final_r05/bench.json 2> gpurun_out/final_r05/bench.log; rc=$?
echo "bench rc=$rc"; tail -4 gpurun_out/final_r05/bench.log; [ $rc -eq 0 ] || exit $rc
FULL=1 bash scripts/evidence.sh r05f_cornell || exit 1
bash scripts/evidence_all.sh r05f sphere c256 mc0.3
