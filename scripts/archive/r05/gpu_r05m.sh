#!/usr/bin/env bash
# Round 5: the 192 MB theta table (x >= 0 on the 2^-23 grid) against the 256 MB one (variant
# libpt_hip_thfull.so, the previous build), config 3 (modified Cornell r = 0, 0.3, 0.8), after
# the GPU suite on the new build.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R"
V="PT_LIB=$R/pathtracer-cpp_amd/lib/variants/libpt_hip_thfull.so"
A="--scene mcornell --rough 0 --spp 3000"; B="--scene mcornell --rough 0.3 --spp 3000"; C="--scene mcornell --rough 0.8 --spp 3000"
bash scripts/ab.sh \
  "m0_half||$A" "m0_full|$V|$A" "m3_half||$B" "m3_full|$V|$B" "m8_half||$C" "m8_full|$V|$C" \
  "m0_half2||$A" "m0_full2|$V|$A" "m3_half2||$B" "m3_full2|$V|$B" "m8_half2||$C" "m8_full2|$V|$C"
