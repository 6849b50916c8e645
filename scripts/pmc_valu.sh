#!/usr/bin/env bash
# VALU issue per ray of bench variants (one PMC pass each, kernel-only single step):
# main-port slots (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2), all VALU instructions and
# lane utilisation per traced ray of the trace kernel. Section costs by difference against
# PT_EXP_DUP_* builds (a section executed twice).
# usage: bash scripts/pmc_valu.sh TAG "NAME|ENV=VAL ...|bench args" ...  -> gpurun_out/pmcv_TAG/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$R/gpurun_out/pmcv_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r name envs args <<< "$spec"
  envs="${envs//@R@/$R}"  # @R@: the repository root on the box (absolute library paths)
  timeout -s KILL 300 env PT_TEST_HOOKS=1 $envs rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 \
    SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE -d "$OUT/$name" -o sq --output-format csv -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e $args > "$OUT/$name.json" 2> "$OUT/$name.log" \
    || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  python3 - "$OUT" "$name" <<'PY'
import csv, glob, json, sys, collections
out, name = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(float)
for f in glob.glob(f"{out}/{name}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "trace" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
b = json.loads(open(f"{out}/{name}.json").read().strip().splitlines()[-1])
rays = b["rays_per_step"]
main = (acc["SQ_ACTIVE_INST_VALU"] - acc["SQ_ACTIVE_INST_VALU2"]) / rays
insts = acc["SQ_INSTS_VALU"] / rays
lanes = acc["SQ_THREAD_CYCLES_VALU"] / max(acc["SQ_ACTIVE_INST_VALU"], 1) / 64
print(f"{name:14s} main-port/ray {main:7.3f}  valu/ray {insts:7.3f}  lanes {lanes:.3f}  "
      f"kernel {b['kernel_mrays']:.0f} Mray/s  rays {rays:.4g}")
PY
done
