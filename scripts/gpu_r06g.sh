#!/usr/bin/env bash
# Round 6: the cold frame's table kernel with the scene's flags (path 5) — GPU suite, speed,
# cold end to end.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06g
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06g/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06g/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash scripts/ab.sh "fast|PT_RTC=0|--spp 3000 --no-e2e" "gen|PT_RTC=0 PT_FLAT_FAST=0|--spp 3000 --no-e2e" \
  "mfast|PT_RTC=0|--scene mcornell --spp 3000 --no-e2e" "mgen|PT_RTC=0 PT_FLAT_FAST=0|--scene mcornell --spp 3000 --no-e2e" || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06g/e2e_$i.json 2> gpurun_out/r06g/e2e_$i.log || exit 1
  grep "end to end" gpurun_out/r06g/e2e_$i.log
done
PT_TEST_HOOKS=1 PT_FLAT_FAST=0 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06g/e2e_gen.json 2> gpurun_out/r06g/e2e_gen.log || exit 1
grep "end to end" gpurun_out/r06g/e2e_gen.log
