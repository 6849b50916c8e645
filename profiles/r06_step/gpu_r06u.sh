#!/usr/bin/env bash
# Round 6: what a headline step spends outside the trace kernels (whole job 0.5 % below
# kernel-only): kernel + memory-copy trace of one timed frame, every event and gap listed.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/r06u"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/r06u/kt" -o kt --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > "$R/gpurun_out/r06u/b.json" 2> "$R/gpurun_out/r06u/b.log" || { echo "trace failed"; tail -5 "$R/gpurun_out/r06u/b.log"; exit 1; }
cd "$R" && python3 - <<'PY'
import csv, glob
ev = []
for kind in ("kernel_trace", "memory_copy_trace"):
    for f in glob.glob("gpurun_out/r06u/kt/**/*%s.csv" % kind, recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or ("copy " + r.get("Direction", "")) 
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:60]))
ev.sort()
# the timed frame: the events after the last trace kernel of the warm-up frame; print the last 30
tail = ev[-30:]
t0 = tail[0][0]; prev = None
busy = 0
for s, e, n in tail:
    gap = (s - prev) / 1e6 if prev else 0.0
    busy += e - s
    print("  +%9.3f ms  %9.3f ms  gap %8.3f  %s" % ((s - t0) / 1e6, (e - s) / 1e6, gap, n))
    prev = e
print("span %.3f ms busy %.3f ms" % ((tail[-1][1] - t0) / 1e6, busy / 1e6))
PY
