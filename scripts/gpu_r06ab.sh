#!/usr/bin/env bash
# Round 6: the separate pass over a sample-major flagged slab (one-launch frames: an 8-GPU share)
# gathering 128 samples' bits and up to 8 records a step, against the previous build (variant
# libpt_hip_prevacc.so): GPU suite, the headline's and config 4's share, config 4's frame, and a
# kernel trace of the share's step.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ab/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06ab/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
V="$R/pathtracer-cpp_amd/lib/variants/libpt_hip_prevacc.so"
SKIP_TESTS=1 bash scripts/ab.sh "p8_new||--part 0/8 --steps 5 --no-e2e" "p8_prev|PT_LIB=$V|--part 0/8 --steps 5 --no-e2e" \
  "p8_new2||--part 0/8 --steps 5 --no-e2e" "p8_prev2|PT_LIB=$V|--part 0/8 --steps 5 --no-e2e" \
  "c4p8_new||--scene sphere --spp 1000 --part 0/8 --steps 5 --no-e2e" "c4p8_prev|PT_LIB=$V|--scene sphere --spp 1000 --part 0/8 --steps 5 --no-e2e" \
  "c4_new||--scene sphere --spp 1000 --steps 3 --no-e2e" "c4_prev|PT_LIB=$V|--scene sphere --spp 1000 --steps 3 --no-e2e" \
  "fw_new||--steps 3 --no-e2e" "fw_prev|PT_LIB=$V|--steps 3 --no-e2e" || exit 1
bash scripts/gpu_r06aa.sh
