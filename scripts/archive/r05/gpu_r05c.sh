#!/usr/bin/env bash
# Round 5: the dark-path skip of the unwinding (PT_DARK_SKIP) and sparse slabs - GPU suite,
# A/B: sparse (default) / dark skip with every record stored (PT_SPARSE=0) / neither (PT_DARK=0)
# on configs 2, 3 (r = 0.3), 4 and 5 (1024^2 d8 here),
# then config 4's section split by duplication (scripts/gpu_r05b.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash scripts/ab.sh \
  "cor_sparse||--spp 2000" "cor_dark|PT_SPARSE=0|--spp 2000" "cor_full|PT_DARK=0|--spp 2000" \
  "c4_sparse||--scene sphere --spp 1000" "c4_dark|PT_SPARSE=0|--scene sphere --spp 1000" "c4_full|PT_DARK=0|--scene sphere --spp 1000" \
  "mc03_sparse||--scene mcornell --rough 0.3 --spp 2000" "mc03_dark|PT_SPARSE=0|--scene mcornell --rough 0.3 --spp 2000" "mc03_full|PT_DARK=0|--scene mcornell --rough 0.3 --spp 2000" \
  "d8_sparse||--depth 8 --spp 1000" "d8_dark|PT_SPARSE=0|--depth 8 --spp 1000" "d8_full|PT_DARK=0|--depth 8 --spp 1000" \
  "cor_sparse2||--spp 2000" "cor_dark2|PT_SPARSE=0|--spp 2000" "cor_full2|PT_DARK=0|--spp 2000" \
  "c4_sparse2||--scene sphere --spp 1000" "c4_dark2|PT_SPARSE=0|--scene sphere --spp 1000" "c4_full2|PT_DARK=0|--scene sphere --spp 1000" || exit 1
bash scripts/gpu_r05b.sh
