#!/usr/bin/env bash
# Round 6: guided refills, cached gather buffers, slab release — GPU suite, A/B, part balance,
# compile timing on the box's host.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06d/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rtc_timing.py > gpurun_out/r06d/rtc_timing.jsonl 2>&1; echo "rtc_timing rc=$?"; cat gpurun_out/r06d/rtc_timing.jsonl
S="--scene sphere --spp 1000 --no-e2e"
SKIP_TESTS=1 bash scripts/ab.sh "c4_g||$S" "c4_ng|PT_GUIDED=0|$S" "cor_g||--spp 3000 --no-e2e" "cor_ng|PT_GUIDED=0|--spp 3000 --no-e2e" \
  "c4_g2||$S" "c4_ng2|PT_GUIDED=0|$S" "cor_g2||--spp 3000 --no-e2e" "cor_ng2|PT_GUIDED=0|--spp 3000 --no-e2e" || exit 1
timeout -k 10 300 python3 scripts/part_balance.py --scene sphere --res 1024 --spp 1000 --depth 5 --band 1 --ns 8 > gpurun_out/r06d/bal_c4_g.json 2> gpurun_out/r06d/bal_c4_g.log; echo "bal g rc=$?"
PT_TEST_HOOKS=1 PT_GUIDED=0 timeout -k 10 300 python3 scripts/part_balance.py --scene sphere --res 1024 --spp 1000 --depth 5 --band 1 --ns 8 > gpurun_out/r06d/bal_c4_ng.json 2> gpurun_out/r06d/bal_c4_ng.log; echo "bal ng rc=$?"
python3 - <<'PY'
import json
for f in ("gpurun_out/r06d/bal_c4_g.json", "gpurun_out/r06d/bal_c4_ng.json"):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(f, "unreadable", e); continue
    q = d["partitions"]["8"]
    print(f, "whole %.1f ms kernel %.1f" % (d["whole"]["wall_ms"], d["whole"]["kernel_ms"]), "worst/ideal %.4f kernel %.4f" % (q["worst_over_ideal"], q["worst_kernel_over_ideal"]),
          "parts", [round(t["kernel_ms"], 2) for t in q["parts"]], "rays ok", q["rays_sum_equals_whole"])
PY
