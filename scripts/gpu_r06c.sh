#!/usr/bin/env bash
# Round 6: the whole GPU suite with the compile server, exit races on the GPU, one bench line.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06c/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06c/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash scripts/exit_race.sh 20 > gpurun_out/r06c/exit_race.log 2>&1; echo "exit_race rc=$?"; tail -1 gpurun_out/r06c/exit_race.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r06c/bench.json 2> gpurun_out/r06c/bench.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06c/bench.log; exit $rc; }
python3 -c "import json; d=json.loads(open('gpurun_out/r06c/bench.json').read().strip().splitlines()[-1]); e=d.get('end_to_end',{}); print('value', round(d['value']), 'kernel', round(d['kernel_mrays']), 'e2e', {k: e.get(k) for k in ('value','seconds','first_frame_s','warm','device_init_s')})"
