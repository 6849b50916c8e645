#!/usr/bin/env bash
# Round 4: hipRTC flat kernel under other LLVM scheduler settings (same arithmetic, so the
# same bits; parity checked for the chosen one): AMDGPU register-pressure trackers at 7 and
# 8 waves (62 / 63 VGPRs, no scratch), max-ILP strategy, post-RA machine scheduling.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04j
run() {  # name, env..., -- bench args
  local name=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 300 env PT_TEST_HOOKS=1 "${envs[@]}" python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e "$@" \
    > gpurun_out/r04j/$name.json 2> gpurun_out/r04j/$name.log || { echo "$name failed"; tail -5 gpurun_out/r04j/$name.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r04j/$name.json')); print('$name', 'Mray/s=%.0f'%d['value'], 'kernel_mrays=%.0f'%d['kernel_mrays'])"
}
TR="PT_RTC_FLAGS=-mllvm -amdgpu-use-amdgpu-trackers"
TR8="PT_RTC_WAVES=8"
ILP="PT_RTC_FLAGS=-mllvm -amdgpu-sched-strategy=gcn-max-ilp"
POST="PT_RTC_FLAGS=-mllvm -misched-postra"
timeout -k 10 300 env PT_TEST_HOOKS=1 "$TR" PT_RTC_WAVES=8 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "vs_oracle or golden_images or albedo_x2" > gpurun_out/r04j/pytest_tr8.log 2>&1; rc=$?
echo "pytest tr8 rc=$rc"; tail -2 gpurun_out/r04j/pytest_tr8.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  run cor_base$rep -- --spp 1000
  run cor_tr$rep "$TR" -- --spp 1000
  run cor_tr8_$rep "$TR" "$TR8" -- --spp 1000
  run cor_ilp$rep "$ILP" -- --spp 1000
  run cor_post$rep "$POST" -- --spp 1000
done
run mc_base PT_RTC_WAVES=7 -- --scene mcornell --rough 0.3 --spp 1000
run mc_tr "$TR" -- --scene mcornell --rough 0.3 --spp 1000
run mc_tr8 "$TR" "$TR8" -- --scene mcornell --rough 0.3 --spp 1000
run c5_base PT_RTC_WAVES=7 -- --res 4096 --depth 8 --spp 64
run c5_tr8 "$TR" "$TR8" -- --res 4096 --depth 8 --spp 64
