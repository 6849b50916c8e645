#!/usr/bin/env bash
# Round 4 checkpoint: the whole GPU suite, smoke(), and the default bench line (with the
# cold and warm-cache end-to-end passes and the CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/chk
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/chk/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/chk/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/chk/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/chk/bench.json 2> gpurun_out/chk/bench.log; rc=$?
echo "bench rc=$rc"; tail -4 gpurun_out/chk/bench.log; exit $rc
