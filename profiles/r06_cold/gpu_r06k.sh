#!/usr/bin/env bash
# Round 6: threaded scene packing + 64-refill pool default — GPU suite, cold end to end (config 4 x3,
# headline x2), config 4's N = 8 share at R = 64 / 128 / 256 refills, and the scene kernel compiled
# at -O2 (compile time vs kernel speed: kernel-only pairs, cold lines).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06k/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06k/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene sphere --spp 1000 > gpurun_out/r06k/e2e_c4_$i.json 2> gpurun_out/r06k/e2e_c4_$i.log || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06k/e2e_$i.json 2> gpurun_out/r06k/e2e_$i.log || exit 1
  PT_TEST_HOOKS=1 PT_RTC_FLAGS="-O2 -fno-slp-vectorize" timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06k/e2e_o2_$i.json 2> gpurun_out/r06k/e2e_o2_$i.log || exit 1
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06k/e2e*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); e = d["end_to_end"]
    print(f, "cold %.0f Mray/s (%.3f s) kernel-only %.0f ratio %.3f build %.3f set_scene %.3f s frame %.3f s" % (e["value"], e["seconds"], d["kernel_mrays"], e["value"] / d["kernel_mrays"], e["bvh_build_s"], e["set_scene_s"], e["frame_with_d2h_s"]))
PY
for rf in 64 128 256 64b; do
  PT_TEST_HOOKS=1 PT_POOL_REFILLS=${rf%b} timeout -k 10 300 python3 scripts/part_balance.py --scene sphere --res 1024 --spp 1000 --depth 5 --band 1 --ns 8 > gpurun_out/r06k/bal_c4_r$rf.json 2> gpurun_out/r06k/bal_c4_r$rf.log || { echo "bal $rf failed"; exit 1; }
done
python3 - <<'PY'
import json
for rf in ("64", "128", "256", "64b"):
    d = json.load(open("gpurun_out/r06k/bal_c4_r%s.json" % rf)); q = d["partitions"]["8"]
    print("refills", rf, "whole %.1f ms kernel %.1f" % (d["whole"]["wall_ms"], d["whole"]["kernel_ms"]), "worst/ideal %.4f kernel %.4f" % (q["worst_over_ideal"], q["worst_kernel_over_ideal"]),
          "parts", [round(t["kernel_ms"], 2) for t in q["parts"]], "rays ok", q["rays_sum_equals_whole"])
PY
SKIP_TESTS=1 bash scripts/ab.sh "cor_o3||--spp 3000 --no-e2e" "cor_o2|PT_RTC_FLAGS=-O2,-fno-slp-vectorize|--spp 3000 --no-e2e" \
  "cor_o3b||--spp 3000 --no-e2e" "cor_o2b|PT_RTC_FLAGS=-O2,-fno-slp-vectorize|--spp 3000 --no-e2e" \
  "mc_o3||--scene mcornell --rough 0.3 --spp 2000 --no-e2e" "mc_o2|PT_RTC_FLAGS=-O2,-fno-slp-vectorize|--scene mcornell --rough 0.3 --spp 2000 --no-e2e"
