#!/usr/bin/env bash
# Round 5: two triangle-queue entries per enqueue iteration in the wide step (PT_WIDE_ENQ2=1,
# the flat kernel's form) against one (variants built from the same sources), config 4.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R"
V="PT_LIB=$R/pathtracer-cpp_amd/lib/variants/libpt_hip"
A="--scene sphere --spp 1000"
SKIP_TESTS=1 bash scripts/ab.sh "e1|${V}_enq1.so|$A" "e2|${V}_enq2.so|$A" "e1b|${V}_enq1.so|$A" "e2b|${V}_enq2.so|$A" \
  "e1c|${V}_enq1.so|$A" "e2c|${V}_enq2.so|$A"
