# N>1 rehearsal at HEAD on one GPU: torchrun (2 and 4 ranks) and bench.py's own spawn (2 ranks), collectives on gloo
set -u
cd $GRAFT_REPO_ROOT
bash scripts/rehearse_dist.sh "2 4" --spp 1000 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
PT_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --spp 1000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/reh/spawn2.json 2> gpurun_out/reh/spawn2.log || { echo spawn failed; tail -5 gpurun_out/reh/spawn2.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/reh/spawn2.json')); w=d['world']; print('spawn2', round(d['value']), w['world_size'], w['backend'], w['launcher'], [r['rows'] for r in w['ranks']])"
