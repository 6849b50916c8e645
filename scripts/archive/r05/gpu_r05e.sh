#!/usr/bin/env bash
# Round 5, third box: the GPU suite on the current build (flat sign-bit mask off, no
# pt_scene_prepare), config 4's while-while threshold re-tuned after the dark-path skip
# (PT_WIDE_THRESH 20/24/28/32/36), the default bench line (cold and warm end to end).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
A="--scene sphere --spp 1000"
SKIP_TESTS=1 bash scripts/ab.sh "t28||$A" "t20|PT_WIDE_THRESH=20|$A" "t24|PT_WIDE_THRESH=24|$A" \
  "t32|PT_WIDE_THRESH=32|$A" "t36|PT_WIDE_THRESH=36|$A" "t28b||$A" "t24b|PT_WIDE_THRESH=24|$A" "t32b|PT_WIDE_THRESH=32|$A" || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.log; rc=$?
echo "bench rc=$rc"; tail -3 $O/bench.log; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$O/bench.json')); e=d['end_to_end']; print('headline', d['value'], 'e2e', e['value'], 'warm', (e.get('warm') or {}).get('value'), 'ctx', e['context_create_s'], 'frame', e['frame_with_d2h_s'])"
bash scripts/dropin_e2e.sh || exit 1
bash scripts/gpu_r05f.sh
