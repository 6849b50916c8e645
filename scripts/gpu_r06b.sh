#!/usr/bin/env bash
# Round 6: PMC of config 4 with binary16 planes (6 waves) and float planes (5 waves: no spills).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
W5="$R/pathtracer-cpp_amd/lib/variants/libpt_hip_w5.so"
S="--scene sphere --spp 1000"
bash scripts/pmc_ab.sh r06_planes "f16||$S" "f32w5|PT_WIDE_PLANES=f32 PT_LIB=$W5|$S" "f16w5|PT_LIB=$W5|$S"
