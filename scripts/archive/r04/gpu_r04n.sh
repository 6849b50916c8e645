#!/usr/bin/env bash
# Round 4: knob re-tuning at 8 waves (gpu_r04m.sh), then the keyed PMC evidence of the
# current build for all ten config workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash scripts/gpu_r04m.sh || exit $?
bash scripts/evidence_all.sh r04
