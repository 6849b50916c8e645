#!/usr/bin/env bash
# Round 6, final build (flag layout by frame): one bench line per config (scripts/configs.sh r06b,
# each with its CPU baseline and end-to-end pass), config 4's and the headline's 8-GPU share
# balance, and the GPU suite.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06bal2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06bal2/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06bal2/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for extra in "" "PT_POOL_CHUNK=64 PT_TEST_HOOKS=1"; do
  timeout -k 10 300 env $extra python bench.py --spp 40 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/r06bal2/spp40.json 2> gpurun_out/r06bal2/spp40.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r06bal2/spp40.json')); print('spp40 [$extra] whole %.0f kernel %.0f launch %.3f ms' % (d['value'], d['kernel_mrays'], d['roofline']['avg_launch_ms']))"
done
bash scripts/configs.sh r06b || exit 1
export PT_TEST_HOOKS=1
timeout -k 10 500 python -u scripts/part_balance.py --band 1 --scene cornell --res 1024 --spp 10000 --depth 5 --ns 2 4 8 > gpurun_out/r06bal2/cfg2.json 2> gpurun_out/r06bal2/cfg2.log || exit 1
timeout -k 10 500 python -u scripts/part_balance.py --band 1 --scene sphere --res 1024 --spp 1000 --depth 5 --ns 2 4 8 --reps 2 > gpurun_out/r06bal2/cfg4.json 2> gpurun_out/r06bal2/cfg4.log || exit 1
echo done
