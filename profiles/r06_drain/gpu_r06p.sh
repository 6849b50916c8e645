#!/usr/bin/env bash
# Round 6: the work pool's tail (last refills of a launch from a second counter in chunk / 8
# items) against PT_POOL_TAIL=0: GPU suite, config 4 share fixed cost + 8-GPU balance, the
# headline's per-launch cost (2728 spp in 2 / 4 / 8 launches), whole-frame pairs.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06p/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06p/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
export PT_TEST_HOOKS=1
for tail in 1 0; do
  export PT_POOL_TAIL=$tail
  timeout -k 10 300 python3 scripts/part_tail.py --scene sphere --res 1024 --depth 5 --part 0/8 --spp 250 500 1000 2000 --reps 2 > gpurun_out/r06p/tail_c4_t$tail.json 2> gpurun_out/r06p/tail_c4_t$tail.log || exit 1
  timeout -k 10 300 python3 scripts/part_balance.py --scene sphere --res 1024 --spp 1000 --depth 5 --band 1 --ns 8 > gpurun_out/r06p/bal_c4_t$tail.json 2> gpurun_out/r06p/bal_c4_t$tail.log || exit 1
  for b in 1364 682 341; do
    timeout -k 10 300 python3 scripts/part_tail.py --scene cornell --res 1024 --depth 5 --part 0/1 --spp 2728 --reps 2 --batch $b > gpurun_out/r06p/cor_t${tail}_b$b.json 2> gpurun_out/r06p/cor_t${tail}_b$b.log || exit 1
  done
done
unset PT_POOL_TAIL
python3 - <<'PY'
import json
import numpy as np
for t in ("1", "0"):
    d = json.load(open("gpurun_out/r06p/tail_c4_t%s.json" % t))
    print("tail", t, "c4 part 0/8: %.5f ms/spp, fixed %.3f ms" % (d["ms_per_spp"], d["fixed_ms"]), [(r["spp"], round(min(r["kernel_ms"]), 3)) for r in d["rows"]])
    b = json.load(open("gpurun_out/r06p/bal_c4_t%s.json" % t)); q = b["partitions"]["8"]
    print("tail", t, "c4 N=8 worst/ideal %.4f kernel %.4f whole kernel %.1f ms" % (q["worst_over_ideal"], q["worst_kernel_over_ideal"], b["whole"]["kernel_ms"]), [round(x["kernel_ms"], 2) for x in q["parts"]])
    xs, ys = [], []
    for bb in (1364, 682, 341):
        r = json.load(open("gpurun_out/r06p/cor_t%s_b%d.json" % (t, bb)))["rows"][0]
        xs.append(r["trace_launches"]); ys.append(min(r["kernel_ms"]))
    a, c = np.polyfit(xs, ys, 1)
    print("tail", t, "cornell 2728 spp:", list(zip(xs, [round(y, 3) for y in ys])), "per-launch %.3f ms" % a)
PY
SKIP_TESTS=1 bash scripts/ab.sh "cor_tail||--spp 3000 --no-e2e" "cor_notail|PT_POOL_TAIL=0|--spp 3000 --no-e2e" \
  "c4_tail||--scene sphere --spp 1000 --no-e2e" "c4_notail|PT_POOL_TAIL=0|--scene sphere --spp 1000 --no-e2e" \
  "cor_tail2||--spp 3000 --no-e2e" "cor_notail2|PT_POOL_TAIL=0|--spp 3000 --no-e2e" \
  "c4_tail2||--scene sphere --spp 1000 --no-e2e" "c4_notail2|PT_POOL_TAIL=0|--scene sphere --spp 1000 --no-e2e"
