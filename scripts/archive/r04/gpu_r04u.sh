#!/usr/bin/env bash
# Round 4: the offline 8-wide walk (config 4) with the camera fields from its argument
# registers (variant library, -DPT_CAM_KERNARG=0) against the kernarg-segment default.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
V=$PWD/pathtracer-cpp_amd/lib/variants/libpt_hip_camreg.so
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "s_ka1::--scene sphere" "s_reg1:PT_LIB=$V:--scene sphere" "s_ka2::--scene sphere" "s_reg2:PT_LIB=$V:--scene sphere" \
  "s_ka3::--scene sphere" "s_reg3:PT_LIB=$V:--scene sphere"
