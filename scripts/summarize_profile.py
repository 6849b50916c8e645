#!/usr/bin/env python3
"""Summarise a gpurun_out/ev_<tag> evidence directory (scripts/evidence.sh) into
profiles/<tag>/<workload>/ and the keyed per-workload PMC file bench.py reads.

Per dispatch of the dominant kernel (the trace kernel): average duration from the
kernel trace (checked against the bench's own HIP-event average), HBM traffic =
FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts half of a wide streaming read,
MI355X_MICROARCH.md §HBM) + WRITE_SIZE (rocprofv3 reports KiB), and the SQ
instruction / lane-utilisation / wait counters, all per ray and per launch.
profiles/pmc/<scene>_<W>x<H>_depth<d>.json carries the kernel key (sha256 of the
kernel sources, bench.py: kernel_key) the pass was taken with; bench.py ignores it
for any other build.
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


def is_trace(name):
    return "pt_trace_kernel" in name or "pt_trace_flat_rtc" in name


def kname(n):
    return "trace" if is_trace(n) else "accumulate" if "accumulate" in n else n


bench = json.load(open(os.path.join(src, "kt.json")))
cfg = bench["config"]
W, H = cfg["res"]
workload = f"{cfg['scene']}_{W}x{H}_depth{cfg['depth']}"
dst = os.path.join(ROOT, "profiles", tag, workload)
os.makedirs(dst, exist_ok=True)

pmc = collections.defaultdict(float)
dispatches = collections.Counter()
for f in glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = (kname(r["Kernel_Name"]), r["Counter_Name"])
        pmc[k] += float(r["Counter_Value"])
        dispatches[k] += 1
stats = {}
for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))):
    stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "pct": float(r["Percentage"])}
trace = [v for k, v in stats.items() if is_trace(k)][0]
# Span from the first trace dispatch's start to the last one's end over the launch count
# (includes the accumulate kernels between launches), beside rocprof's per-dispatch average.
starts, ends = [], []
for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_trace.csv"))):
    if is_trace(r["Kernel_Name"]):
        starts.append(int(r["Start_Timestamp"]))
        ends.append(int(r["End_Timestamp"]))
span_ns = (max(ends) - min(starts)) if starts else 0
rays_step = bench["rays_per_step"]
launches = trace["calls"]
rays_launch = rays_step / launches


def per_launch(counter):
    return pmc.get(("trace", counter), 0.0) / max(dispatches.get(("trace", counter), 1), 1)


VALU_MAIN_PEAK = 256 * 4 * 2.4e9 / 4  # main-port slots/s: 4 cycles per wave64 VALU instruction at 2.4 GHz
t_launch_s = trace["avg_ns"] * 1e-9
main_slots = per_launch("SQ_ACTIVE_INST_VALU") - per_launch("SQ_ACTIVE_INST_VALU2")
fetch = per_launch("FETCH_SIZE") * 1024 * 2
write = per_launch("WRITE_SIZE") * 1024
valu = per_launch("SQ_INSTS_VALU")
waves_cyc = per_launch("SQ_WAVE_CYCLES")
t = {
    "avg_duration_ms": trace["avg_ns"] / 1e6,
    "span_per_launch_ms": span_ns / 1e6 / max(len(starts), 1),
    "bench_hip_event_avg_launch_ms": bench["roofline"]["avg_launch_ms"],
    "launches_per_frame": launches,
    "rays_per_launch": rays_launch,
    "hbm_read_bytes_fetchx2": fetch,
    "hbm_write_bytes": write,
    "hbm_bytes_per_ray": (fetch + write) / rays_launch,
    "algorithmic_bytes_per_ray": bench["hbm_algorithmic"]["bytes_per_ray"],
    "valu_insts_per_ray": valu / rays_launch,
    "salu_insts_per_ray": per_launch("SQ_INSTS_SALU") / rays_launch,
    "lds_insts_per_ray": per_launch("SQ_INSTS_LDS") / rays_launch,
    "valu_lane_utilisation": per_launch("SQ_THREAD_CYCLES_VALU") / max(64 * per_launch("SQ_ACTIVE_INST_VALU"), 1),
    "wait_any_frac": per_launch("SQ_WAIT_ANY") / max(waves_cyc, 1),
    "wait_inst_any_frac": per_launch("SQ_WAIT_INST_ANY") / max(waves_cyc, 1),
    "l2_hit_rate": per_launch("TCC_HIT_sum") / max(per_launch("TCC_HIT_sum") + per_launch("TCC_MISS_sum"), 1),
    # VALU main-port issue (calibrated by tools/valu_ubench): every wave-instruction
    # occupies the SIMD's main VALU port for 4 cycles (transcendentals 8: SQ_ACTIVE_INST_VALU
    # counts them twice) unless it was issued on the second port (SQ_ACTIVE_INST_VALU2: simple
    # VOP1/VOP2-class f32 add/sub/mul and integer add/and/mov dual-issue there).
    "valu_main_slots_per_ray": main_slots / rays_launch,
    "valu_second_port_slots_per_ray": per_launch("SQ_ACTIVE_INST_VALU2") / rays_launch,
    "valu_main_port_frac": main_slots / (t_launch_s * VALU_MAIN_PEAK),
    "gpu_clock_ghz_grbm": per_launch("GRBM_GUI_ACTIVE") / 8 / t_launch_s / 1e9 if per_launch("GRBM_GUI_ACTIVE") else None,
    "valu_insts_issue_frac_2cyc_model": valu / t_launch_s / (256 * 4 * 2.4e9 / 2),
}
summary = {
    "tag": tag,
    "workload": workload,
    "bench_cmd": "python bench.py " + " ".join(sys.argv[2:]) if len(sys.argv) > 2 else bench["config"]["workload"],
    "kernel_key": bench["roofline"]["pmc_key"],
    "bench_value_mrays": bench["value"],
    "kernel_stats": stats,
    "trace_kernel_per_dispatch": t,
    "pmc_per_dispatch_raw": {f"{k[0]}:{k[1]}": v / max(dispatches[k], 1) for k, v in sorted(pmc.items())},
}
json.dump(summary, open(os.path.join(dst, "profile_summary.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
if os.path.exists(os.path.join(src, "bench.json")):
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
os.makedirs(os.path.join(ROOT, "profiles", "pmc"), exist_ok=True)
json.dump({"workload": workload, "key": bench["roofline"]["pmc_key"],
           "valu_insts_per_ray": t["valu_insts_per_ray"], "valu_lane_utilisation": t["valu_lane_utilisation"],
           "valu_main_slots_per_ray": t["valu_main_slots_per_ray"],
           "valu_second_port_slots_per_ray": t["valu_second_port_slots_per_ray"],
           "hbm_bytes_per_ray": t["hbm_bytes_per_ray"], "wait_any_frac": t["wait_any_frac"],
           "gpu_clock_ghz_grbm": t["gpu_clock_ghz_grbm"],
           "source": f"profiles/{tag}/{workload}/profile_summary.json"},
          open(os.path.join(ROOT, "profiles", "pmc", workload + ".json"), "w"), indent=1)
print(json.dumps(t, indent=1))
