#!/usr/bin/env bash
# Keyed PMC evidence for every config workload (scripts/evidence.sh), one after another.
# usage: bash scripts/evidence_all.sh ROUND [names...]  -> gpurun_out/ev_<ROUND>_<name>/
#        then (here): for each: python scripts/summarize_profile.py <ROUND>_<name>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
ROUND=$1; shift
declare -A W=(
  [cornell]=""
  [sphere]="--scene sphere --spp 1000"
  [mc0]="--scene mcornell --rough 0"
  [mc0.05]="--scene mcornell --rough 0.05"
  [mc0.1]="--scene mcornell --rough 0.1"
  [mc0.3]="--scene mcornell --rough 0.3"
  [mc0.5]="--scene mcornell --rough 0.5"
  [mc0.8]="--scene mcornell --rough 0.8"
  [c256]="--res 256 --spp 16 --depth 3"
  [c4096]="--res 4096 --depth 8"
)
NAMES=("$@")
[ ${#NAMES[@]} -eq 0 ] && NAMES=(cornell sphere mc0 mc0.05 mc0.1 mc0.3 mc0.5 mc0.8 c256 c4096)
for n in "${NAMES[@]}"; do
  bash "$R/scripts/evidence.sh" "${ROUND}_$n" ${W[$n]} || { echo "evidence $n failed"; exit 1; }
done
