#!/usr/bin/env bash
# Round 5 end, part C: keyed PMC evidence for the remaining workloads (scripts/evidence_all.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash scripts/evidence_all.sh r05f mc0 mc0.05 mc0.1 mc0.5 mc0.8 c4096
