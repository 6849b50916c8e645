#!/usr/bin/env bash
# Round 5, second box: the VALU issue microbenchmark (1/2/4/8 waves per SIMD), config 4's
# section split by duplication (scripts/gpu_r05b.sh), the drop-in modified_cornell timing
# (fresh vs cached contexts), and the keyed rocprofv3 evidence of the headline (Cornell) and
# config-4 (sphere) kernels (scripts/evidence.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash scripts/gpu_r05_ubench.sh || exit 1
bash scripts/dropin_timing.sh || exit 1
bash scripts/gpu_r05b.sh || exit 1
bash scripts/evidence_all.sh r05 cornell sphere || exit 1
