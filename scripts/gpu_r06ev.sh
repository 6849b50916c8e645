#!/usr/bin/env bash
# Round 6 final build: keyed PMC evidence for every config workload (scripts/evidence_all.sh).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && bash scripts/evidence_all.sh "$@"
