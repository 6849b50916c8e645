mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --spp 1000 --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.log; rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench_quick.log; cat gpurun_out/bench_quick.json
exit $rc
