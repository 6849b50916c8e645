#!/usr/bin/env bash
# Round 4: camera fields in argument registers (default now) vs the kernarg segment
# (PT_CAM_KERNARG=1): VALU slots per ray (keyed-free PMC) and more timing pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
K=PT_RTC_DEFINES=PT_CAM_KERNARG=1
bash scripts/pmc_valu.sh cam "c_reg||--spp 1000" "c_ka|$K|--spp 1000" \
  "m_reg||--scene mcornell --rough 0.3 --spp 1000" "m_ka|$K|--scene mcornell --rough 0.3 --spp 1000" || exit 1
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "m_reg1::--scene mcornell --rough 0.3 --spp 1000" "m_ka1:$K:--scene mcornell --rough 0.3 --spp 1000" \
  "m_reg2::--scene mcornell --rough 0.3 --spp 1000" "m_ka2:$K:--scene mcornell --rough 0.3 --spp 1000" \
  "m_reg3::--scene mcornell --rough 0.3 --spp 1000" "m_ka3:$K:--scene mcornell --rough 0.3 --spp 1000" \
  "c_reg1::--spp 1000" "c_ka1:$K:--spp 1000" "m8_reg::--scene mcornell --rough 0.8 --spp 1000" \
  "m8_ka:$K:--scene mcornell --rough 0.8 --spp 1000"
