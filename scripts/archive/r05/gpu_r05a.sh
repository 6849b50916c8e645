#!/usr/bin/env bash
# Round 5, first box: the whole GPU suite (albedo-x2 overflow cases, cached device contexts,
# origins on box planes, dark-path skip, sparse slabs), A/B of the sign-bit box masks
# (hipRTC flat kernel: PT_RTC_DEFINES=PT_SIGN_MASK=0; wide walk: the variant library built with
# -DPT_SIGN_MASK=0) and of the dark-path skip / sparse slabs (PT_SPARSE=0: every record
# stored; PT_DARK=0: every path unwound), then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
NS="PT_LIB=$PWD/pathtracer-cpp_amd/lib/variants/libpt_hip_dup_nosign.so"
SKIP_TESTS=1 bash scripts/ab.sh \
  "c4_sign||--scene sphere --spp 1000" "c4_nosign|$NS|--scene sphere --spp 1000" \
  "cor_sign||--spp 1500" "cor_nosign|PT_RTC_DEFINES=PT_SIGN_MASK=0|--spp 1500" \
  "cor_dark|PT_SPARSE=0|--spp 1500" "cor_full|PT_DARK=0|--spp 1500" \
  "c4_dark|PT_SPARSE=0|--scene sphere --spp 1000" "c4_full|PT_DARK=0|--scene sphere --spp 1000" \
  "mc03_sign||--scene mcornell --rough 0.3 --spp 1500" "mc03_nosign|PT_RTC_DEFINES=PT_SIGN_MASK=0|--scene mcornell --rough 0.3 --spp 1500" \
  "mc03_full|PT_DARK=0|--scene mcornell --rough 0.3 --spp 1500" \
  "c4_sign2||--scene sphere --spp 1000" "c4_nosign2|$NS|--scene sphere --spp 1000" \
  "cor_sign2||--spp 1500" "cor_nosign2|PT_RTC_DEFINES=PT_SIGN_MASK=0|--spp 1500" \
  "cor_dark2|PT_SPARSE=0|--spp 1500" "cor_full2|PT_DARK=0|--spp 1500" || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.log; rc=$?
echo "bench rc=$rc"; tail -3 $O/bench.log; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$O/bench.json')); print('headline', d['value'], d.get('end_to_end',{}).get('value'))"
