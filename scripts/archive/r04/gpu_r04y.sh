#!/usr/bin/env bash
# Round 4: the scene kernel compiled at -O2 / -O1 instead of -O3 (PT_RTC_FLAGS, appended:
# the last -O wins): kernel speed, hipRTC compile time, cold end to end.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/r04y
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "o3::--spp 1000" "o2:PT_RTC_FLAGS=-O2:--spp 1000" "o1:PT_RTC_FLAGS=-O1:--spp 1000" \
  "o3b::--spp 1000" "o2b:PT_RTC_FLAGS=-O2:--spp 1000" "o1b:PT_RTC_FLAGS=-O1:--spp 1000" \
  "mo3::--scene mcornell --rough 0.3 --spp 1000" "mo2:PT_RTC_FLAGS=-O2:--scene mcornell --rough 0.3 --spp 1000" || exit 1
cat > /tmp/rtct.py <<'PY'
import sys, time, ctypes as C, os
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "pathtracer-cpp_amd"))
os.environ["PT_RTC_CACHE"] = "0"
import ptamd
from ptamd import scenes
ref = ptamd._SceneRef(ptamd.BVH.from_scene(scenes.cornell((8, 8))))
t = time.perf_counter(); ptamd.lib().pt_rtc_check(C.byref(ref.s), None, 0); print("%.3f" % (time.perf_counter() - t))
PY
export GRAFT_REPO_ROOT=$PWD
for f in "" "-O2" "-O1"; do
  echo "compile '$f': $(for i in 1 2 3; do PT_TEST_HOOKS=1 PT_RTC_FLAGS="$f" timeout -k 10 120 python /tmp/rtct.py; done | tr '\n' ' ')"
done
for spec in "e3:" "e2:-O2" "e1:-O1" "e3b:" "e2b:-O2"; do
  n=${spec%%:*}; f=${spec#*:}
  timeout -k 10 300 env PT_TEST_HOOKS=1 PT_RTC_FLAGS="$f" python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04y/$n.json 2> gpurun_out/r04y/$n.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04y/$n.json'))['end_to_end']; print('$n', 'cold %.0f'%d['value'], 'frame %.3f'%d['frame_with_d2h_s'], 'warm %.0f'%d['warm']['value'])"
done
