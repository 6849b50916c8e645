#!/usr/bin/env bash
# GPU test suite + a short headline bench + the --gpus N guard on a 1-GPU box.
# usage: bash scripts/archive/r03/gpu_tests_r03.sh TAG -> gpurun_out/t_TAG/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/t_$1"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=6 -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python bench.py --gpus 2 --steps 1 --warmup 0 > "$OUT/bench_gpus2.json" 2> "$OUT/bench_gpus2.log"; echo "gpus2 rc=$? (2 expected)"; tail -2 "$OUT/bench_gpus2.log"
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.log"; rc2=$?
echo "bench rc=$rc2"; tail -c 1500 "$OUT/bench.json"
exit $rc
