#!/usr/bin/env bash
# Round 6: after removing the pool tail — GPU suite; with the scaled step bar, config 4's 8-GPU
# share at 64 and 128 refills per wave (balance x2 each, share fixed cost) and whole-frame pairs.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06q
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06q/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06q/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
export PT_TEST_HOOKS=1
for rf in 64 128 64b 128b; do
  export PT_POOL_REFILLS=${rf%b}
  timeout -k 10 300 python3 scripts/part_balance.py --scene sphere --res 1024 --spp 1000 --depth 5 --band 1 --ns 8 > gpurun_out/r06q/bal_c4_r$rf.json 2> gpurun_out/r06q/bal_c4_r$rf.log || exit 1
done
for rf in 64 128; do
  export PT_POOL_REFILLS=$rf
  timeout -k 10 300 python3 scripts/part_tail.py --scene sphere --res 1024 --depth 5 --part 0/8 --spp 250 500 1000 2000 --reps 2 > gpurun_out/r06q/tail_c4_r$rf.json 2> gpurun_out/r06q/tail_c4_r$rf.log || exit 1
done
unset PT_POOL_REFILLS
python3 - <<'PY'
import json
for rf in ("64", "128", "64b", "128b"):
    b = json.load(open("gpurun_out/r06q/bal_c4_r%s.json" % rf)); q = b["partitions"]["8"]
    print("R", rf, "c4 N=8 worst/ideal %.4f kernel %.4f whole kernel %.1f ms" % (q["worst_over_ideal"], q["worst_kernel_over_ideal"], b["whole"]["kernel_ms"]), [round(x["kernel_ms"], 2) for x in q["parts"]])
for rf in ("64", "128"):
    d = json.load(open("gpurun_out/r06q/tail_c4_r%s.json" % rf))
    print("R", rf, "c4 part 0/8: %.5f ms/spp, fixed %.3f ms" % (d["ms_per_spp"], d["fixed_ms"]), [(r["spp"], round(min(r["kernel_ms"]), 3)) for r in d["rows"]])
PY
SKIP_TESTS=1 bash scripts/ab.sh "c4_r64||--scene sphere --spp 1000 --no-e2e" "c4_r128|PT_POOL_REFILLS=128|--scene sphere --spp 1000 --no-e2e" \
  "cor_r64||--spp 3000 --no-e2e" "cor_r128|PT_POOL_REFILLS=128|--spp 3000 --no-e2e"
