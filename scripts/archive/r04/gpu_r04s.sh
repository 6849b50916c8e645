#!/usr/bin/env bash
# Round 4: the whole GPU suite on the final scene-kernel defaults, then the keyed PMC
# evidence of the final kernel sources.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04s
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r04s/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r04s/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/evidence_all.sh r04
