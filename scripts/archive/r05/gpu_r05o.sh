#!/usr/bin/env bash
# Round 5: the GPU suite with an option forced on for every test (robustness of the non-default
# paths across all scenes and kernels): sparse slabs everywhere, the fused accumulation's tail
# batch, box-level pairs, the dark-path skip off. Tests that assert the default itself are
# expected to fail under an override; the log lists them.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/forced
for spec in "sparse:PT_SPARSE=1" "tail:PT_TAIL_DIV=4" "box:PT_BOX_PAIRS=1" "nodark:PT_DARK=0"; do
  name="${spec%%:*}"; envs="${spec#*:}"
  timeout -k 10 400 env PT_TEST_HOOKS=1 $envs python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/forced/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; grep -E "passed|failed" gpurun_out/forced/$name.log | tail -1; grep "^FAILED" gpurun_out/forced/$name.log | head -8
  [ $rc -le 1 ] || exit $rc
done
