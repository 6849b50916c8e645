#!/usr/bin/env bash
# Round 6: flag words pixel-major per 32 samples (one load per 32 samples in the accumulation)
# against the round-5 layout (variant libpt_hip_oldflags.so): GPU suite; headline whole frame x2,
# the headline's and config 4's 8-GPU share (--part 0/8, one launch + the separate pass), config 5.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "flag or dark or tail or refill or full_size or golden or oracle or progressive or multi_batch" > gpurun_out/r06x_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06x_pytest.log; [ $rc -eq 0 ] || exit $rc
V="$R/pathtracer-cpp_amd/lib/variants/libpt_hip_oldflags.so"
SKIP_TESTS=1 bash scripts/ab.sh "fw_new||--steps 3 --no-e2e" "fw_old|PT_LIB=$V|--steps 3 --no-e2e" \
  "fw_new2||--steps 3 --no-e2e" "fw_old2|PT_LIB=$V|--steps 3 --no-e2e" \
  "p8_new||--part 0/8 --steps 5 --no-e2e" "p8_old|PT_LIB=$V|--part 0/8 --steps 5 --no-e2e" \
  "p8_new2||--part 0/8 --steps 5 --no-e2e" "p8_old2|PT_LIB=$V|--part 0/8 --steps 5 --no-e2e" \
  "c4p8_new||--scene sphere --spp 1000 --part 0/8 --steps 5 --no-e2e" "c4p8_old|PT_LIB=$V|--scene sphere --spp 1000 --part 0/8 --steps 5 --no-e2e" \
  "c5_new||--res 4096 --depth 8 --steps 1 --no-e2e" "c5_old|PT_LIB=$V|--res 4096 --depth 8 --steps 1 --no-e2e"
