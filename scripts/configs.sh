#!/usr/bin/env bash
# One bench line per BASELINE.json config on one GPU, each with its CPU baseline (the
# unmodified reference, one core, bounded sample) and the end-to-end pass:
#   cfg1 Cornell 256^2 16 spp d3 (its CPU baseline is the whole config)
#   cfg2 Cornell 1024^2 10k spp d5 (headline)
#   cfg3 modified Cornell 1024^2 10k spp d5, roughness 0, 0.05, 0.1, 0.3, 0.5, 0.8
#   cfg4 99k-triangle sphere mesh 1024^2 1k spp d5
#   cfg5 Cornell 4096^2 10k spp d8 (the 8-GPU config, here on one GPU)
# usage: bash scripts/configs.sh TAG [cfg names...]   -> gpurun_out/configs_TAG/*.json
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$R/gpurun_out/configs_$TAG"; mkdir -p "$OUT"
cd "$R"
declare -A C=(
  [cfg1_cornell256]="--res 256 --spp 16 --depth 3 --steps 5 --warmup 2 --cpu-spp 16"
  [cfg2_cornell1024]="--steps 3 --warmup 1"
  [cfg3_mcornell_r0]="--scene mcornell --rough 0 --steps 1 --warmup 1"
  [cfg3_mcornell_r0.05]="--scene mcornell --rough 0.05 --steps 1 --warmup 1"
  [cfg3_mcornell_r0.1]="--scene mcornell --rough 0.1 --steps 1 --warmup 1"
  [cfg3_mcornell_r0.3]="--scene mcornell --rough 0.3 --steps 1 --warmup 1"
  [cfg3_mcornell_r0.5]="--scene mcornell --rough 0.5 --steps 1 --warmup 1"
  [cfg3_mcornell_r0.8]="--scene mcornell --rough 0.8 --steps 1 --warmup 1"
  [cfg4_sphere]="--scene sphere --spp 1000 --steps 3 --warmup 1"
  [cfg5_cornell4096_d8]="--res 4096 --depth 8 --steps 1 --warmup 0 --cpu-spp 1"
)
NAMES=("$@")
if [ ${#NAMES[@]} -eq 0 ]; then NAMES=($(printf '%s\n' "${!C[@]}" | sort)); fi
for n in "${NAMES[@]}"; do
  timeout -k 10 600 python3 bench.py ${C[$n]} > "$OUT/$n.json" 2> "$OUT/$n.log" || { echo "$n failed"; tail -5 "$OUT/$n.log"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d.get('cpu_baseline') or {}; e=d.get('end_to_end') or {}; print('%-22s %9.0f Mray/s  e2e %9.0f  cpu %6.2f Mray/s (%s)' % (sys.argv[2], d['value'], e.get('value', 0), c.get('value', 0), c.get('kind')))" "$OUT/$n.json" "$n"
done
