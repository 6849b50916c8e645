# Headline at 20 steps (the driver's shape) and one rank's share at N = 2, 4, 8 timed alone (final kernels)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/long
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/long/steps20.json 2> gpurun_out/long/steps20.log || { echo bench failed; tail -3 gpurun_out/long/steps20.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/long/steps20.json')); print('steps20', round(d['value']), round(d['ms_per_step'],2), d['roofline']['frac'])"
for p in 0/2 0/4 0/8 7/8; do
  n=$(echo $p | tr / _)
  timeout -k 10 300 python bench.py --part $p --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/long/part$n.json 2> gpurun_out/long/part$n.log || { echo part failed; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('part', sys.argv[2], round(d['ms_per_step'],2), 'ms')" gpurun_out/long/part$n.json $p
done
