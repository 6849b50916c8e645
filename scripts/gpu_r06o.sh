#!/usr/bin/env bash
# Round 6: the wide step loop's bar scaled by the lanes holding paths (product) against the fixed
# bar (variant libpt_hip_thrfixed.so): GPU suite, config 4 share fixed cost and 8-GPU balance,
# whole-frame kernel-only pairs; and the flat kernel's per-launch cost on the headline (one
# frame of 2728 spp in 1, 2, 4 and 8 launches).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06o
V="$R/pathtracer-cpp_amd/lib/variants/libpt_hip_thrfixed.so"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06o/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06o/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for lib in product fixed; do
  if [ $lib = fixed ]; then export PT_LIB="$V"; else unset PT_LIB; fi
  timeout -k 10 300 python3 scripts/part_tail.py --scene sphere --res 1024 --depth 5 --part 0/8 --spp 250 500 1000 2000 --reps 2 > gpurun_out/r06o/tail_c4_$lib.json 2> gpurun_out/r06o/tail_c4_$lib.log || exit 1
  timeout -k 10 300 python3 scripts/part_balance.py --scene sphere --res 1024 --spp 1000 --depth 5 --band 1 --ns 8 > gpurun_out/r06o/bal_c4_$lib.json 2> gpurun_out/r06o/bal_c4_$lib.log || exit 1
done
unset PT_LIB
python3 - <<'PY'
import json
for lib in ("product", "fixed"):
    d = json.load(open("gpurun_out/r06o/tail_c4_%s.json" % lib))
    print(lib, "c4 part 0/8: %.5f ms/spp, fixed %.3f ms" % (d["ms_per_spp"], d["fixed_ms"]), [(r["spp"], round(min(r["kernel_ms"]), 3)) for r in d["rows"]])
    b = json.load(open("gpurun_out/r06o/bal_c4_%s.json" % lib)); q = b["partitions"]["8"]
    print(lib, "c4 N=8 worst/ideal %.4f kernel %.4f whole kernel %.1f ms" % (q["worst_over_ideal"], q["worst_kernel_over_ideal"], b["whole"]["kernel_ms"]), [round(t["kernel_ms"], 2) for t in q["parts"]])
PY
SKIP_TESTS=1 bash scripts/ab.sh "c4_scaled||--scene sphere --spp 1000 --no-e2e" "c4_fixed|PT_LIB=$V|--scene sphere --spp 1000 --no-e2e" \
  "c4_scaled2||--scene sphere --spp 1000 --no-e2e" "c4_fixed2|PT_LIB=$V|--scene sphere --spp 1000 --no-e2e" || exit 1
for b in 2728 1364 682 341; do
  timeout -k 10 300 python3 scripts/part_tail.py --scene cornell --res 1024 --depth 5 --part 0/1 --spp 2728 --reps 2 --batch $b > gpurun_out/r06o/cor_b$b.json 2> gpurun_out/r06o/cor_b$b.log || exit 1
done
python3 - <<'PY'
import json
import numpy as np
xs, ys = [], []
for b in (2728, 1364, 682, 341):
    d = json.load(open("gpurun_out/r06o/cor_b%d.json" % b)); r = d["rows"][0]
    xs.append(r["trace_launches"]); ys.append(min(r["kernel_ms"]))
    print("cornell 2728 spp batch %d: %d launches, kernel %.3f ms" % (b, r["trace_launches"], min(r["kernel_ms"])))
a, t = np.polyfit(xs, ys, 1)
print("cornell per-launch cost %.3f ms (frame %.1f ms at 1 launch)" % (a, t + a))
PY
