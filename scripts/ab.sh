#!/usr/bin/env bash
# GPU A/B timing: optional GPU parity tests, then one bench line per variant.
# usage: bash scripts/ab.sh "NAME|ENV=VAL ENV2=VAL|bench args" ...   (SKIP_TESTS=1 to skip pytest)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/ab
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/ab/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
for spec in "$@"; do
  IFS='|' read -r name envs args <<< "$spec"
  timeout -k 10 300 env PT_TEST_HOOKS=1 $envs python bench.py --steps 1 --warmup 1 --no-cpu-baseline $args > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "bench $name rc=$rc"; tail -5 gpurun_out/ab/$name.log; exit $rc; fi
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-12s %9.0f Mray/s  kernel %9.0f Mray/s  %s' % (sys.argv[2], d['value'], d['kernel_mrays'], d['roofline']['kernel']))" gpurun_out/ab/$name.json $name
done
