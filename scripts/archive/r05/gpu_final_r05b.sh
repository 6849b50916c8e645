#!/usr/bin/env bash
# Round 5 end, part B: one bench line per BASELINE.json config (scripts/configs.sh r05).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash scripts/configs.sh r05
