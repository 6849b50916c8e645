#!/usr/bin/env bash
# Round 4: flat pair queues shortened where one more block per CU then fits the LDS (the
# default now) — the whole GPU suite, A/B against 512-entry queues (PT_PAIR_QUEUE=512), then
# the keyed PMC evidence and the round-end rehearsal with config lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04ac
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r04ac/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r04ac/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
Q=PT_PAIR_QUEUE=512
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "m_new::--scene mcornell --rough 0.3 --spp 1000" "m_512:$Q:--scene mcornell --rough 0.3 --spp 1000" \
  "m_newb::--scene mcornell --rough 0.3 --spp 1000" "m_512b:$Q:--scene mcornell --rough 0.3 --spp 1000" \
  "m8_new::--scene mcornell --rough 0.8 --spp 1000" "m8_512:$Q:--scene mcornell --rough 0.8 --spp 1000" \
  "s_new::--res 4096 --depth 8 --spp 64" "s_512:$Q:--res 4096 --depth 8 --spp 64" \
  "s_newb::--res 4096 --depth 8 --spp 64" "s_512b:$Q:--res 4096 --depth 8 --spp 64" \
  "c_new::--spp 1000" "c_512:$Q:--spp 1000" || exit $?
bash scripts/evidence_all.sh r04 || exit $?
bash scripts/gpu_final_r04.sh
