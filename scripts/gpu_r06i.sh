#!/usr/bin/env bash
# Round 6: switch to the scene kernel at the first launch boundary after its compile; cold e2e.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06i/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06i/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06i/e2e_$i.json 2> gpurun_out/r06i/e2e_$i.log || exit 1
  grep "end to end" gpurun_out/r06i/e2e_$i.log
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene sphere --spp 1000 > gpurun_out/r06i/e2e_c4_$i.json 2> gpurun_out/r06i/e2e_c4_$i.log || exit 1
  grep "end to end" gpurun_out/r06i/e2e_c4_$i.log
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06i/e2e*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); e = d["end_to_end"]
    print(f, "cold %.0f Mray/s (%.3f s) kernel-only %.0f ratio %.3f set_scene %.3f s frame %.3f s" % (e["value"], e["seconds"], d["kernel_mrays"], e["value"] / d["kernel_mrays"], e["set_scene_s"], e["frame_with_d2h_s"]))
PY
