#!/usr/bin/env bash
# Round 6: flag bit layout chosen per render (pixel-major for frames of several launches, with
# up to 8 records in flight in the separate pass; sample-major for one-launch frames) against the
# round-5 layout (variant libpt_hip_oldflags.so): the flag tests, then whole frames and 8-GPU
# shares of the headline and config 4, config 5.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06y
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06y/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06y/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
V="$R/pathtracer-cpp_amd/lib/variants/libpt_hip_oldflags.so"
SKIP_TESTS=1 bash scripts/ab.sh "fw_new||--steps 3 --no-e2e" "fw_old|PT_LIB=$V|--steps 3 --no-e2e" \
  "p8_new||--part 0/8 --steps 5 --no-e2e" "p8_old|PT_LIB=$V|--part 0/8 --steps 5 --no-e2e" \
  "p8_pm|PT_FLAGS_PM=1|--part 0/8 --steps 5 --no-e2e" \
  "fw_new2||--steps 3 --no-e2e" "fw_old2|PT_LIB=$V|--steps 3 --no-e2e" \
  "p8_new2||--part 0/8 --steps 5 --no-e2e" "p8_old2|PT_LIB=$V|--part 0/8 --steps 5 --no-e2e" \
  "p8_pm2|PT_FLAGS_PM=1|--part 0/8 --steps 5 --no-e2e" \
  "c4p8_new||--scene sphere --spp 1000 --part 0/8 --steps 5 --no-e2e" "c4p8_old|PT_LIB=$V|--scene sphere --spp 1000 --part 0/8 --steps 5 --no-e2e" \
  "c4_new||--scene sphere --spp 1000 --steps 3 --no-e2e" "c4_old|PT_LIB=$V|--scene sphere --spp 1000 --steps 3 --no-e2e" \
  "c5_new||--res 4096 --depth 8 --steps 1 --no-e2e" "c5_old|PT_LIB=$V|--res 4096 --depth 8 --steps 1 --no-e2e"
