#!/usr/bin/env bash
# Round 6: flat table grouped by flat axis; cold end to end; -O2 for the scene kernel (A/B).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06h/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06h/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
O2="PT_RTC_FLAGS=-O2,-fno-slp-vectorize"
SKIP_TESTS=1 bash scripts/ab.sh "fast|PT_RTC=0|--spp 3000 --no-e2e" "gen|PT_RTC=0 PT_FLAT_FAST=0|--spp 3000 --no-e2e" \
  "mfast|PT_RTC=0|--scene mcornell --spp 3000 --no-e2e" \
  "m3|$O2|--scene mcornell --spp 3000 --no-e2e" "m3o3||--scene mcornell --spp 3000 --no-e2e" \
  "c5o2|$O2|--res 4096 --depth 8 --spp 300 --no-e2e" "c5o3||--res 4096 --depth 8 --spp 300 --no-e2e" \
  "m8|$O2|--scene mcornell --rough 0.8 --spp 3000 --no-e2e" "m8o3||--scene mcornell --rough 0.8 --spp 3000 --no-e2e" || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06h/e2e_$i.json 2> gpurun_out/r06h/e2e_$i.log || exit 1
  grep "end to end" gpurun_out/r06h/e2e_$i.log
done
for i in 1 2; do
  PT_TEST_HOOKS=1 PT_RTC_FLAGS=-O2,-fno-slp-vectorize timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06h/e2e_o2_$i.json 2> gpurun_out/r06h/e2e_o2_$i.log || exit 1
  grep "end to end" gpurun_out/r06h/e2e_o2_$i.log
done
