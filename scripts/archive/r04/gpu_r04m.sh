#!/usr/bin/env bash
# Round 4: the scene kernel's runtime knobs re-tuned at 8 waves: camera-ray regeneration
# threshold, pair-phase priority, theta-table lane threshold (config 3).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "cor::--spp 1000" "cor_rg16:PT_REGEN_THRESH=16:--spp 1000" "cor_rg24:PT_REGEN_THRESH=24:--spp 1000" \
  "cor_rg40:PT_REGEN_THRESH=40:--spp 1000" "cor_rg48:PT_REGEN_THRESH=48:--spp 1000" \
  "cor_prio0:PT_RTC_DEFINES=PT_PRIO_PAIRS=0:--spp 1000" "cor_fold1:PT_RTC_DEFINES=PT_PRIO_FOLD=1:--spp 1000" \
  "cor2::--spp 1000" \
  "mc::--scene mcornell --rough 0.3 --spp 1000" "mc_th16:PT_THETA_LANES=16:--scene mcornell --rough 0.3 --spp 1000" \
  "mc_th48:PT_THETA_LANES=48:--scene mcornell --rough 0.3 --spp 1000" "mc_rg24:PT_REGEN_THRESH=24:--scene mcornell --rough 0.3 --spp 1000" \
  "mc_rg40:PT_REGEN_THRESH=40:--scene mcornell --rough 0.3 --spp 1000" "mc2::--scene mcornell --rough 0.3 --spp 1000"
# the one scheduler option that still changes the scene kernel's code with the trackers on
mkdir -p gpurun_out
for n in cor_unclus cor_unclus2; do
  timeout -k 10 300 env PT_TEST_HOOKS=1 "PT_RTC_FLAGS=-mllvm -amdgpu-disable-unclustered-high-rp-reschedule" python bench.py \
    --steps 1 --warmup 1 --spp 1000 --no-cpu-baseline --no-e2e > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); print('$n', 'Mray/s=%.0f'%d['value'], 'kernel_mrays=%.0f'%d['kernel_mrays'])"
done
SKIP_TESTS=1 bash scripts/gpu_ab.sh "cor3::--spp 1000"
