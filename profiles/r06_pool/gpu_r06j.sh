#!/usr/bin/env bash
# Round 6: GPU suite, cold end to end (headline x3, config 4 x2), then config 4's N = 8 share
# balance against the work-pool refill size (PT_POOL_REFILLS: refills per wave the size aims at).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06j
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06j/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06j/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06j/e2e_$i.json 2> gpurun_out/r06j/e2e_$i.log || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene sphere --spp 1000 > gpurun_out/r06j/e2e_c4_$i.json 2> gpurun_out/r06j/e2e_c4_$i.log || exit 1
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06j/e2e*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); e = d["end_to_end"]
    print(f, "cold %.0f Mray/s (%.3f s) kernel-only %.0f ratio %.3f set_scene %.3f s frame %.3f s" % (e["value"], e["seconds"], d["kernel_mrays"], e["value"] / d["kernel_mrays"], e["set_scene_s"], e["frame_with_d2h_s"]))
PY
for rf in 4 64 16 32 4b 64b; do
  PT_TEST_HOOKS=1 PT_POOL_REFILLS=${rf%b} timeout -k 10 300 python3 scripts/part_balance.py --scene sphere --res 1024 --spp 1000 --depth 5 --band 1 --ns 8 > gpurun_out/r06j/bal_c4_r$rf.json 2> gpurun_out/r06j/bal_c4_r$rf.log || { echo "bal $rf failed"; exit 1; }
done
python3 - <<'PY'
import json
for rf in ("4", "64", "16", "32", "4b", "64b"):
    d = json.load(open("gpurun_out/r06j/bal_c4_r%s.json" % rf)); q = d["partitions"]["8"]
    print("refills", rf, "whole %.1f ms kernel %.1f" % (d["whole"]["wall_ms"], d["whole"]["kernel_ms"]), "worst/ideal %.4f kernel %.4f" % (q["worst_over_ideal"], q["worst_kernel_over_ideal"]),
          "parts", [round(t["kernel_ms"], 2) for t in q["parts"]], "rays ok", q["rays_sum_equals_whole"])
PY
SKIP_TESTS=1 bash scripts/ab.sh "c4_r4||--scene sphere --spp 1000 --no-e2e" "c4_r64|PT_POOL_REFILLS=64|--scene sphere --spp 1000 --no-e2e" "cor_r4||--spp 3000 --no-e2e" "cor_r64|PT_POOL_REFILLS=64|--spp 3000 --no-e2e"
