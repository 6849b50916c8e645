#!/usr/bin/env bash
# Round 6: where a 1364-spp batch loses whole-job time against the default 682 (kernel-only
# +0.9 %, whole job -1.1 %): kernel + memory-copy trace of one timed frame each.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/r06s"
cd /tmp && export TMPDIR=/tmp
for b in 1364 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$R/gpurun_out/r06s/kt_b$b" -o kt --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --batch $b > "$R/gpurun_out/r06s/b$b.json" 2> "$R/gpurun_out/r06s/b$b.log" || { echo "trace b$b failed"; tail -5 "$R/gpurun_out/r06s/b$b.log"; exit 1; }
done
cd "$R" && python3 - <<'PY'
import csv, glob
for b in ("1364", "0"):
    ev = []
    for kind in ("kernel_trace", "memory_copy_trace"):
        fs = glob.glob("gpurun_out/r06s/kt_b%s/**/*%s.csv" % (b, kind), recursive=True)
        if not fs:
            continue
        for r in csv.DictReader(open(fs[0])):
            name = r.get("Kernel_Name") or r.get("Direction") or kind
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:50]))
    ev.sort()
    # the last frame: from the last trace kernel launch group; print the final 40 events
    print("batch", b, "events", len(ev))
    tail = ev[-45:]
    t0 = tail[0][0]
    prev = None
    for s, e, n in tail:
        gap = (s - prev) / 1e6 if prev else 0.0
        print("  +%9.3f ms  %8.3f ms  gap %7.3f  %s" % ((s - t0) / 1e6, (e - s) / 1e6, gap, n))
        prev = e
PY
