#!/usr/bin/env bash
# PMC passes (one rocprofv3 --pmc run per counter group) over a short bench run.
# usage: bash scripts/pmc.sh TAG "C1 C2 ..." ["C3 ..."] ...   (BENCH_ARGS env overrides the bench args)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$R/gpurun_out/pmc_$TAG"; mkdir -p "$OUT"
read -r -a BA <<< "${BENCH_ARGS:---steps 1 --warmup 0 --spp 400 --no-cpu-baseline}"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  read -r -a CS <<< "$grp"
  timeout -k 10 300 rocprofv3 --pmc "${CS[@]}" -d "$OUT/p$i" -o p$i --output-format csv -- \
      python3 "$R/bench.py" "${BA[@]}" > "$OUT/p$i.json" 2> "$OUT/p$i.log" || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]; agg = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(out + "/p*/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1] + ":" + r["Counter_Name"]
        agg[k] += float(r["Counter_Value"]); n[k] += 1
res = {k: {"sum": v, "dispatches": n[k]} for k, v in sorted(agg.items()) if "pt_" in k}
json.dump(res, open(out + "/summary.json", "w"), indent=1)
for k, v in res.items(): print(k, "%.4g" % v["sum"], v["dispatches"])
PY
