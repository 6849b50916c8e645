#!/usr/bin/env python3
"""Summarise a gpurun_out/ev_<tag> evidence directory into profiles/<tag>/.

Per dispatch of the dominant kernel (pt_trace_kernel): average duration from the
kernel trace, HBM traffic = FETCH_SIZE * 2 (gfx950: FETCH_SIZE counts half of a
wide streaming read, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB units of
rocprofv3, and the SQ instruction / lane-utilisation counters.
usage: python scripts/summarize_profile.py TAG
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src = os.path.join(ROOT, "gpurun_out", f"ev_{tag}")
dst = os.path.join(ROOT, "profiles", tag)
os.makedirs(dst, exist_ok=True)


def kname(r):
    n = r["Kernel_Name"]
    return "pt_trace_kernel" if ("pt_trace_kernel" in n or "pt_trace_flat_rtc" in n) else \
        "pt_accumulate_kernel" if "accumulate" in n else n


pmc = collections.defaultdict(lambda: [0.0, 0])
for f in glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = (kname(r), r["Counter_Name"])
        pmc[k][0] += float(r["Counter_Value"])
        pmc[k][1] += 1
per = {f"{k[0]}:{k[1]}": v[0] / v[1] for k, v in pmc.items() if k[0].startswith("pt_")}
stats = {}
for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))):
    stats[kname({"Kernel_Name": r["Name"]})] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                                "pct": float(r["Percentage"])}
bench = json.load(open(os.path.join(src, "kt.json")))
rays_per_launch = bench["roofline"]["rays_per_launch"]
t = "pt_trace_kernel"
fetch = per.get(f"{t}:FETCH_SIZE", 0.0) * 1024 * 2
write = per.get(f"{t}:WRITE_SIZE", 0.0) * 1024
summary = {
    "tag": tag,
    "bench_cmd": "python bench.py --steps 1 --warmup 0 --no-cpu-baseline (Cornell 1024^2, 10k spp, depth 5)",
    "kernel_stats": stats,
    "trace_kernel_per_dispatch": {
        "avg_duration_ms": stats[t]["avg_ns"] / 1e6,
        "rays": rays_per_launch,
        "hbm_read_bytes_fetchx2": fetch,
        "hbm_write_bytes": write,
        "hbm_bytes": fetch + write,
        "hbm_bytes_per_ray": (fetch + write) / rays_per_launch,
        "algorithmic_bytes_per_ray": bench["roofline"]["bytes_per_ray"],
        "valu_insts_per_ray": per.get(f"{t}:SQ_INSTS_VALU", 0) / rays_per_launch,
        "salu_insts_per_ray": per.get(f"{t}:SQ_INSTS_SALU", 0) / rays_per_launch,
        "lds_insts_per_ray": per.get(f"{t}:SQ_INSTS_LDS", 0) / rays_per_launch,
        "valu_lane_utilisation": per.get(f"{t}:SQ_THREAD_CYCLES_VALU", 0) /
                                 max(64 * per.get(f"{t}:SQ_ACTIVE_INST_VALU", 1), 1),
        "wait_any_frac": per.get(f"{t}:SQ_WAIT_ANY", 0) / max(per.get(f"{t}:SQ_WAVE_CYCLES", 1), 1),
        "wait_inst_any_frac": per.get(f"{t}:SQ_WAIT_INST_ANY", 0) / max(per.get(f"{t}:SQ_WAVE_CYCLES", 1), 1),
    },
    "pmc_per_dispatch_raw": per,
}
json.dump(summary, open(os.path.join(dst, "profile_summary.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
if os.path.exists(os.path.join(src, "bench.json")):
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
# per-ray HBM bytes for bench.py's roofline.traffic
json.dump({"config": "cornell_1024_d5", "hbm_bytes_per_ray": (fetch + write) / rays_per_launch,
           "valu_insts_per_ray": per.get(f"{t}:SQ_INSTS_VALU", 0) / rays_per_launch,
           "source": f"profiles/{tag}/profile_summary.json"},
          open(os.path.join(ROOT, "profiles", "pmc_trace_bytes_per_ray.json"), "w"), indent=1)
print(json.dumps(summary["trace_kernel_per_dispatch"], indent=1))
