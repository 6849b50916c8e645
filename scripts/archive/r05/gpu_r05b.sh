#!/usr/bin/env bash
# Round 5: where config 4's issue slots and idle lanes go, by duplication:
# one PMC pass per variant library (lib/variants/libpt_hip_dup_<s>.so: section <s> executed
# twice, its copy kept live), config 4 (99k mesh, 1024^2, 1000 spp, depth 5) kernel-only.
# Section cost = variant - base (main-port slots per ray); section lane utilisation =
# delta SQ_THREAD_CYCLES_VALU / (64 x delta SQ_ACTIVE_INST_VALU).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
A="--scene sphere --spp 1000"
S=()
for v in base node tri cam brdf fold scan enq stack drainq shade; do
  S+=("$v|PT_LIB=@R@/pathtracer-cpp_amd/lib/variants/libpt_hip_dup_$v.so|$A")
done
S+=("prod||$A")
bash scripts/pmc_valu.sh r05_c4dup "${S[@]}"
