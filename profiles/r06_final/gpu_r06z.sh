#!/usr/bin/env bash
# Round 6 final check: the driver's commands on the final build — smoke(), then the bench line
# exactly as the driver runs it (N = 1, 20 steps, 5 warm-up).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06z
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06z/smoke.log 2>&1 || { tail -20 gpurun_out/r06z/smoke.log; exit 1; }
tail -2 gpurun_out/r06z/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06z/bench.json 2> gpurun_out/r06z/bench.log || { tail -20 gpurun_out/r06z/bench.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06z/bench.json").read().strip().splitlines()[-1])
r = d["roofline"]; e = d["end_to_end"]; c = d["cpu_baseline"]
print("value %.0f kernel %.0f frac %s (%s) traffic %s launch %.2f ms" % (d["value"], d["kernel_mrays"], r["frac"], r.get("pmc_key"), r.get("traffic"), r["avg_launch_ms"]))
print("cold %.0f (%.3f s) warm %s cpu %.2f %s bitexact %s" % (e["value"], e["seconds"], (e.get("warm") or {}).get("value"), c["value"], c["kind"], c.get("bitexact_vs_gpu")))
PY
