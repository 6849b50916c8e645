#!/usr/bin/env bash
# Round 4: camera fields from the kernarg segment (default) or the argument registers, at
# 8 waves, three pairs each on configs 2 and 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D=PT_RTC_DEFINES=PT_CAM_KERNARG=0
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "c_ka1::--spp 1000" "c_reg1:$D:--spp 1000" "c_ka2::--spp 1000" "c_reg2:$D:--spp 1000" "c_ka3::--spp 1000" "c_reg3:$D:--spp 1000" \
  "m_ka1::--scene mcornell --rough 0.3 --spp 1000" "m_reg1:$D:--scene mcornell --rough 0.3 --spp 1000" \
  "m_ka2::--scene mcornell --rough 0.3 --spp 1000" "m_reg2:$D:--scene mcornell --rough 0.3 --spp 1000" \
  "s_ka::--res 4096 --depth 8 --spp 64" "s_reg:$D:--res 4096 --depth 8 --spp 64"
