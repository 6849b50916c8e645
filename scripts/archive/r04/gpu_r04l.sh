#!/usr/bin/env bash
# Round 4: the offline 8-wide walk (config 4) under other LLVM scheduler settings
# (variant libraries: AMDGPU pressure trackers, max-ILP strategy), A/B twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
V=$PWD/pathtracer-cpp_amd/lib/variants
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "sph::--scene sphere" "sph_tr:PT_LIB=$V/libpt_hip_tr.so:--scene sphere" "sph_ilp:PT_LIB=$V/libpt_hip_ilp.so:--scene sphere" \
  "sph2::--scene sphere" "sph_tr2:PT_LIB=$V/libpt_hip_tr.so:--scene sphere" "sph_ilp2:PT_LIB=$V/libpt_hip_ilp.so:--scene sphere"
