# Round-end rehearsal at HEAD: the GPU suite, smoke(), and the default bench line
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/final/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/final/smoke.log; exit 1; }
tail -2 gpurun_out/final/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.log || { echo bench failed; tail -5 gpurun_out/final/bench.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/final/bench.json')); print(d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['ms_per_step'])"
