# Quick parity + A/B timing on the GPU box.
# usage: bash scripts/gpu_ab.sh "NAME:ENV=VAL,ENV2=VAL:bench args" ...
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; envs="${rest%%:*}"; args="${rest#*:}"
  envcmd=""; if [ -n "$envs" ]; then envcmd="${envs//,/ }"; fi
  timeout -k 10 300 env PT_TEST_HOOKS=1 $envcmd python bench.py --steps 1 --warmup 1 --spp 1000 --no-cpu-baseline $args > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.log; rc=$?
  if [ $rc -ne 0 ]; then echo "bench $name rc=$rc"; tail -5 gpurun_out/ab_$name.log; exit $rc; fi
  python -c "import json; d=json.load(open('gpurun_out/ab_$name.json')); print('$name', 'Mray/s=%.0f'%d['value'], 'kernel_mrays=%.0f'%d['kernel_mrays'], 'ms/step=%.1f'%d['ms_per_step'])"
done
