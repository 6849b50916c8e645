#!/usr/bin/env bash
# Round 6: 48 GiB slab budget when no compile is pending (16 GiB while one is), halving before
# the 2^31-item bound — GPU suite; headline, config 4 and config 5 against PT_BATCH_BYTES=16 GiB.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06t/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06t/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
G16=17179869184
for spec in "cor|||--steps 3 --warmup 1" "cor16|PT_BATCH_BYTES=$G16||--steps 3 --warmup 1" "corb|||--steps 3 --warmup 1" "cor16b|PT_BATCH_BYTES=$G16||--steps 3 --warmup 1" \
            "c4|||--scene sphere --spp 1000 --steps 3 --warmup 1" "c416|PT_BATCH_BYTES=$G16||--scene sphere --spp 1000 --steps 3 --warmup 1" \
            "c5|||--res 4096 --depth 8 --steps 1 --warmup 1 --no-e2e" "c516|PT_BATCH_BYTES=$G16||--res 4096 --depth 8 --steps 1 --warmup 1 --no-e2e"; do
  IFS='|' read -r name envs _ args <<< "$spec"
  timeout -k 10 300 env PT_TEST_HOOKS=1 $envs python bench.py --no-cpu-baseline $args > gpurun_out/r06t/$name.json 2> gpurun_out/r06t/$name.log || { tail -5 gpurun_out/r06t/$name.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d.get('end_to_end') or {}
w=e.get('warm') if isinstance(e.get('warm'), dict) else {}
print('%-7s whole %.0f kernel %.0f launch %.2f ms step %.2f ms  cold %s warm %s' % (sys.argv[2], d['value'], d['kernel_mrays'], d['roofline']['avg_launch_ms'], d['ms_per_step'],
      '%.0f (%.3f s)' % (e['value'], e['seconds']) if e else '-', '%.0f (%.3f s)' % (w['value'], w['seconds']) if w else '-'))" gpurun_out/r06t/$name.json $name
done
