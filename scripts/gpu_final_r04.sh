#!/usr/bin/env bash
# Round 4 end: the round-end rehearsal (whole GPU suite, smoke(), default bench line) into
# gpurun_out/final, then one bench line per BASELINE.json config (scripts/configs.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/final/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/final/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.log; rc=$?
echo "bench rc=$rc"; tail -4 gpurun_out/final/bench.log; [ $rc -eq 0 ] || exit $rc
bash scripts/configs.sh r04
