#!/usr/bin/env bash
# Round 6: where config 4's 8-GPU share's fixed ~0.7 ms per launch goes — kernel trace of one
# share rendered in 4 launches of 250 spp and in one launch of 1000 spp (per-launch durations:
# a slower first launch = start-up, equal launches = each launch's drain).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/r06m"
cd /tmp && export TMPDIR=/tmp
for b in 250 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r06m/kt_b$b" -o kt --output-format csv -- python3 "$R/scripts/part_tail.py" --scene sphere --res 1024 --depth 5 --part 0/8 --spp 1000 --reps 3 --batch $b > "$R/gpurun_out/r06m/pt_b$b.json" 2> "$R/gpurun_out/r06m/pt_b$b.log" || { echo "trace b$b failed"; tail -5 "$R/gpurun_out/r06m/pt_b$b.log"; exit 1; }
done
cd "$R" && python3 - <<'PY'
import csv, glob
for b in ("250", "0"):
    fs = glob.glob("gpurun_out/r06m/kt_b%s/**/*kernel_trace.csv" % b, recursive=True)
    rows = list(csv.DictReader(open(fs[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    prev_end = None
    print("batch", b)
    for r in rows:
        n = r["Kernel_Name"]
        if "trace" not in n and "flat" not in n and "accum" not in n:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end else 0
        print("  %-40s %9.3f ms  gap before %9.3f ms" % (n[:40], (e - s) / 1e6, gap / 1e3))
        prev_end = e
PY
