#!/usr/bin/env bash
# Round 6: scene-kernel compile time and speed at lower optimisation levels (cold start).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06e
for spec in "o3|" "o2|-O2,-fno-slp-vectorize" "o1|-O1" "o0|-O0"; do
  name="${spec%%|*}"; fl="${spec#*|}"
  PT_TEST_HOOKS=1 PT_RTC_FLAGS="$fl" timeout -k 10 200 python3 scripts/rtc_timing.py > gpurun_out/r06e/rtc_$name.jsonl 2>&1
  echo "$name $(head -1 gpurun_out/r06e/rtc_$name.jsonl)"
done
SKIP_TESTS=1 bash scripts/ab.sh "cor_o3||--spp 3000 --no-e2e" "cor_o2|PT_RTC_FLAGS=-O2,-fno-slp-vectorize|--spp 3000 --no-e2e" \
  "cor_o1|PT_RTC_FLAGS=-O1|--spp 3000 --no-e2e" "cor_gen|PT_RTC=0|--spp 3000 --no-e2e" \
  "mc_o3||--scene mcornell --spp 3000 --no-e2e" "mc_o1|PT_RTC_FLAGS=-O1|--scene mcornell --spp 3000 --no-e2e" \
  "mc_gen|PT_RTC=0|--scene mcornell --spp 3000 --no-e2e"
