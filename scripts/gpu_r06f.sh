#!/usr/bin/env bash
# Round 6: the generic flat kernel (the cold frame's kernel while the scene kernel compiles)
# with Cornell's scene flags baked in (PT_TBL_EXP variants), Cornell, PT_RTC=0.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
V="$R/pathtracer-cpp_amd/lib/variants"
SKIP_TESTS=1 bash scripts/ab.sh "gen|PT_RTC=0|--spp 3000 --no-e2e" "gen_tbl|PT_RTC=0 PT_LIB=$V/libpt_hip_tbl.so|--spp 3000 --no-e2e" \
  "gen_tbl8|PT_RTC=0 PT_LIB=$V/libpt_hip_tbl8.so|--spp 3000 --no-e2e" "gen_tbl8w8|PT_RTC=0 PT_LIB=$V/libpt_hip_tbl8w8.so|--spp 3000 --no-e2e" \
  "gen0|PT_RTC=0|--spp 3000 --no-e2e" "rtc||--spp 3000 --no-e2e"
