#!/usr/bin/env bash
# A/B timing lines: bash scripts/archive/r03/ab_r03.sh TAG "NAME|ENV=VAL ...|bench args" ...  -> gpurun_out/ab_TAG/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$R/gpurun_out/ab_$TAG"; mkdir -p "$OUT"; cd "$R"
for spec in "$@"; do
  IFS='|' read -r name envs args <<< "$spec"
  timeout -k 10 300 env PT_TEST_HOOKS=1 X=1 $envs python3 bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-e2e $args \
    > "$OUT/$name.json" 2> "$OUT/$name.log"; rc=$?
  case $rc in 0) ;; 124|137|134|139) echo "fatal rc=$rc at $name"; exit $rc;; *) echo "bench $name rc=$rc"; tail -3 "$OUT/$name.log"; continue;; esac
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-14s %9.0f Mray/s  kernel %9.0f  launch %.2f ms  launches/step %d' % (sys.argv[2], d['value'], d['kernel_mrays'], d['roofline']['avg_launch_ms'], d['world']['ranks'][0]['trace_launches'] // d['steps']))" "$OUT/$name.json" $name
done
