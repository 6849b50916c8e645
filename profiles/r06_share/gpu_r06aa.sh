#!/usr/bin/env bash
# Round 6: where an 8-GPU headline share's step spends its time outside the trace kernel
# (whole 2.4 % below kernel-only): kernel + memory-copy trace of bench --part 0/8.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/r06aa"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/r06aa/kt" -o kt --output-format csv -- python3 "$R/bench.py" --part 0/8 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > "$R/gpurun_out/r06aa/b.json" 2> "$R/gpurun_out/r06aa/b.log" || { echo "trace failed"; tail -5 "$R/gpurun_out/r06aa/b.log"; exit 1; }
cd "$R" && python3 - <<'PY'
import csv, glob
ev = []
for kind in ("kernel_trace", "memory_copy_trace"):
    for f in glob.glob("gpurun_out/r06aa/kt/**/*%s.csv" % kind, recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or ("copy " + r.get("Direction", ""))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:60]))
ev.sort()
tail = ev[-24:]
t0 = tail[0][0]; prev = None
for s, e, n in tail:
    gap = (s - prev) / 1e6 if prev else 0.0
    print("  +%9.3f ms  %9.3f ms  gap %8.3f  %s" % ((s - t0) / 1e6, (e - s) / 1e6, gap, n))
    prev = e
PY
python3 -c "import json; d=json.loads(open('gpurun_out/r06aa/b.json').read().strip().splitlines()[-1]); print('value %.0f kernel %.0f step %.2f ms' % (d['value'], d['kernel_mrays'], d['ms_per_step']))"
