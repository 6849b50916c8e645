# Quick parity + A/B timing on the GPU box.
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for pi in "$@"; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --spp 1000 --no-cpu-baseline --per-item $pi > gpurun_out/ab_$pi.json 2> gpurun_out/ab_$pi.log; rc=$?
  if [ $rc -ne 0 ]; then echo "bench rc=$rc"; tail -5 gpurun_out/ab_$pi.log; exit $rc; fi
  python -c "import json; d=json.load(open('gpurun_out/ab_$pi.json')); print('per_item=$pi', 'Mray/s=%.0f'%d['value'], 'kernel_mrays=%.0f'%d['kernel_mrays'], 'ms/step=%.1f'%d['ms_per_step'])"
done
