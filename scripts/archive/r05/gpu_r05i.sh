#!/usr/bin/env bash
# Round 5, VERDICT r4 #1's octant-regroup lever, measured as an upper bound on config 4:
# the product build (variant xbase) against builds whose bounce rays are made coherent per
# wave at no cost (PT_EXP_COHERENT_DIR: +-one direction per wave; PT_EXP_OCTANT_DIR: each
# lane's sample moved into the wave's octant where it stays in its hemisphere). Timing twice,
# then one VALU PMC pass each (lanes) and one L2 pass each (TCC hit / miss).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
A="--scene sphere --spp 1000"
V="PT_LIB=$R/pathtracer-cpp_amd/lib/variants/libpt_hip"
SKIP_TESTS=1 bash scripts/ab.sh "base|${V}_xbase.so|$A" "coh|${V}_coh.so|$A" "oct|${V}_oct.so|$A" \
  "base2|${V}_xbase.so|$A" "coh2|${V}_coh.so|$A" "oct2|${V}_oct.so|$A" || exit $?
bash scripts/pmc_valu.sh r05_oct "base|${V}_xbase.so|$A" "coh|${V}_coh.so|$A" "oct|${V}_oct.so|$A" || exit $?
OUT="$R/gpurun_out/pmcl2_r05_oct"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in xbase coh oct; do
  timeout -s KILL 300 env PT_TEST_HOOKS=1 ${V}_$v.so rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
    -d "$OUT/$v" -o l2 --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e $A \
    > "$OUT/$v.json" 2> "$OUT/$v.log" || { echo "l2 $v failed"; tail -5 "$OUT/$v.log"; exit 1; }
  python3 - "$OUT" "$v" <<'PY'
import csv, glob, sys, collections
out, name = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(float)
for f in glob.glob(f"{out}/{name}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "trace" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
h, m = acc["TCC_HIT_sum"], acc["TCC_MISS_sum"]
print(f"{name:8s} L2 hit rate {h / max(h + m, 1):.3f}  hits {h:.4g}  misses {m:.4g}")
PY
done
