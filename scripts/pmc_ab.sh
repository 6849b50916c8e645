#!/usr/bin/env bash
# PMC A/B of bench variants (one SQ pass + one TA/TCP pass each), kernel-only single step.
# usage: bash scripts/pmc_ab.sh TAG "NAME|ENV=VAL ...|bench args" ...  -> gpurun_out/pmc_TAG/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$R/gpurun_out/pmc_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r name envs args <<< "$spec"
  for p in "sq:SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES" \
           "ta:TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
    pn="${p%%:*}"; read -r -a CS <<< "${p#*:}"
    timeout -s KILL 300 env PT_TEST_HOOKS=1 $envs rocprofv3 --pmc "${CS[@]}" -d "$OUT/${name}_$pn" -o "$pn" --output-format csv -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e $args > "$OUT/${name}_$pn.json" 2> "$OUT/${name}_$pn.log" \
      || { echo "$name $pn failed"; tail -5 "$OUT/${name}_$pn.log"; exit 1; }
  done
  python3 - "$OUT" "$name" <<'PY'
import csv, glob, sys, collections
out, name = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(float)
for f in glob.glob(f"{out}/{name}_*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(name, " ".join(f"{k}={v:.4g}" for k, v in sorted(acc.items())))
PY
done
