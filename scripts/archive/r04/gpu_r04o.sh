#!/usr/bin/env bash
# Round 4: the generic flat kernel (first launches of a cold process, PT_RTC=0) with
# distinct leaf boxes + leaf masks against one box per leaf (variant library built from
# the previous sources); then the cold end-to-end headline with each.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
V=$PWD/pathtracer-cpp_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "generic or full_size or vs_oracle" > gpurun_out/r04o_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r04o_pytest.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "gen_new:PT_RTC=0:--spp 1000" "gen_old:PT_RTC=0,PT_LIB=$V/libpt_hip_nodedup.so:--spp 1000" \
  "gen_new2:PT_RTC=0:--spp 1000" "gen_old2:PT_RTC=0,PT_LIB=$V/libpt_hip_nodedup.so:--spp 1000" \
  "mgen_new:PT_RTC=0:--scene mcornell --rough 0.3 --spp 1000" "mgen_old:PT_RTC=0,PT_LIB=$V/libpt_hip_nodedup.so:--scene mcornell --rough 0.3 --spp 1000"
for n in new old new2 old2; do
  lib=""; case $n in old*) lib="PT_LIB=$V/libpt_hip_nodedup.so";; esac
  timeout -k 10 300 env $lib python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/e2e_$n.json 2> gpurun_out/e2e_$n.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/e2e_$n.json'))['end_to_end']; print('e2e_$n', 'cold %.0f'%d['value'], 'frame %.3f'%d['frame_with_d2h_s'], 'warm %.0f'%d['warm']['value'])"
done
