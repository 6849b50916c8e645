#!/usr/bin/env bash
# Round 4 diagnostic: config 4 section counts (stamps) and the BRDF's cost (cheap-libm /
# no-BRDF timing experiments, wrong images) on config 4 and Cornell.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
bash scripts/stamps.sh "sphere|PT_WIDE_THRESH=28|--scene sphere --spp 250" || exit $?
V=pathtracer-cpp_amd/lib/variants
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "sph_base::--scene sphere --spp 1000" \
  "sph_cheap:PT_LIB=$V/libpt_hip_cheaplibm.so:--scene sphere --spp 1000" \
  "sph_nobrdf:PT_LIB=$V/libpt_hip_nobrdf.so:--scene sphere --spp 1000" \
  "cor_base::--spp 1000" \
  "cor_cheap:PT_RTC_DEFINES=PT_EXP_CHEAP_LIBM=1:--spp 1000" \
  "cor_nobrdf:PT_RTC_DEFINES=PT_EXP_NO_BRDF=1:--spp 1000"
