#!/usr/bin/env bash
# Round 5: config 4's "rest" bucket split further by duplication (load offsets, exact leaf-box
# checks, the step loop's exit test, the segment start's 1/d, the claim's item arithmetic),
# one PMC pass each against the base build of the same source.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
A="--scene sphere --spp 1000"
S=()
for v in base offs xbox loopctl start claim; do
  S+=("$v|PT_LIB=@R@/pathtracer-cpp_amd/lib/variants/libpt_hip_dup_$v.so|$A")
done
bash scripts/pmc_valu.sh r05_c4dup2 "${S[@]}"
# the flat (hipRTC) kernel's sections on Cornell the same way (PT_RTC_DEFINES), 2000 spp
C="--spp 2000"
D="PT_RTC_DEFINES"
bash scripts/pmc_valu.sh r05_cordup "base||$C" "mask|$D=PT_EXP_DUP_MASK=1|$C" "pair|$D=PT_EXP_DUP_PAIR=1|$C" \
  "brdf|$D=PT_EXP_DUP_BRDF=1|$C" "camf|$D=PT_EXP_DUP_CAMF=1|$C" "fold|$D=PT_EXP_DUP_FOLD=1|$C"
