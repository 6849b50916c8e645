#!/usr/bin/env python3
"""Summarise the VALU issue calibration into profiles/<tag>/:
tools/valu_ubench under rocprofv3 (kernel trace + SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
SQ_ACTIVE_INST_VALU2, SQ_THREAD_CYCLES_VALU, GRBM_GUI_ACTIVE) -> cycles per wave-instruction
per SIMD and the share issued on the second VALU port, per instruction form; plus the
trace kernels' VALU mix passes (SQ_INSTS_VALU_* and VALU2) -> main-port slots per ray.
usage: python scripts/valu_calibration.py UBENCH_DIR MIX_DIR TAG
  UBENCH_DIR: gpurun_out/<run> holding ub_pmc/, ub_kt/, ubench7.txt (scripts/archive/r03/diag_r03c.sh)
  MIX_DIR:    gpurun_out/<run> holding pmc_{c,s4}_mix{1,2}/ (scripts/archive/r03/diag_r03b.sh)"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["fma", "pk_fma", "pk_mul", "fma_mix", "cvt_ub", "fma_f64", "rcp", "addc", "max3", "add", "mov", "and",
         "cndmask", "cmp", "fma_lo32", "fma_1", "fma_even", "fmac", "mul", "mul_neg", "min", "cndmask_vcc",
         "cndmask_sgpr", "add_u32", "lshl", "cmp_sgpr", "fma+add", "mul+add", "mov_dpp", "sub", "max3+min", "add_abs",
         "fma_2lanes", "fma_4", "fma_16"]


def rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    ub, mix, tag = sys.argv[1:4]
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    by = collections.OrderedDict()
    for r in rows(os.path.join(ub, "ub_pmc")):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0])
        by.setdefault(k, collections.Counter())[r["Counter_Name"]] += float(r["Counter_Value"])
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(ub, "ub_kt", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"].split("(")[0]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    forms, seen = {}, set()
    for (d, n), c in by.items():
        op = int(n.split("<")[1].rstrip(">"))
        if op in seen:
            continue
        seen.add(op)
        ns = min(dur[n])
        per_simd = c["SQ_INSTS_VALU"] / 1024
        clk = c["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9)
        forms[NAMES[op]] = {
            "kernel_ns": ns, "wave_insts_per_simd": round(per_simd),
            "cycles_per_inst_2p4ghz": round(ns * 1e-9 * 2.4e9 / per_simd, 3),
            "cycles_per_inst_grbm_clock": round(ns * 1e-9 * clk / per_simd, 3), "grbm_clock_ghz": round(clk / 1e9, 3),
            "active_valu_per_inst": round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_INSTS_VALU"], 3),
            "second_port_per_inst": round(c["SQ_ACTIVE_INST_VALU2"] / c["SQ_INSTS_VALU"], 3),
            "active_lanes": round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"], 1)}
    kernels = {}
    for sc, label in (("c", "cornell_1024x1024_depth5"), ("s4", "sphere223_in_cornell_1024x1024_depth5")):
        agg = collections.Counter()
        rays = launches = ms = None
        for m in ("mix1", "mix2"):
            for r in rows(os.path.join(mix, f"pmc_{sc}_{m}")):
                if "trace" in r["Kernel_Name"]:
                    agg[r["Counter_Name"]] += float(r["Counter_Value"])
            b = json.load(open(os.path.join(mix, f"pmc_{sc}_{m}.json")))
            rays = b["rays_per_step"]
            launches = rays / b["roofline"]["rays_per_launch"]
            ms = b["roofline"]["avg_launch_ms"]
        per_ray = {k: v / rays for k, v in sorted(agg.items())}
        main = per_ray["SQ_ACTIVE_INST_VALU"] - per_ray["SQ_ACTIVE_INST_VALU2"]
        t = ms * 1e-3 * launches
        kernels[label] = {
            "per_ray": {k: round(v, 4) for k, v in per_ray.items()}, "launches": round(launches),
            "avg_launch_ms": ms, "valu_main_slots_per_ray": round(main, 4),
            "main_port_frac_2p4ghz": round(main * rays / t / (256 * 4 * 2.4e9 / 4), 4),
            "main_port_frac_grbm_clock": round(main * rays / t / (256 * 4 * agg["GRBM_GUI_ACTIVE"] / 8 / t / 4), 4)}
    out = {"ubench": "tools/valu_ubench (7 waves per SIMD, 8 independent chains per wave, 4096 x 8 "
                     "instructions per wave)", "forms": forms, "trace_kernels": kernels}
    json.dump(out, open(os.path.join(dst, "valu_calibration.json"), "w"), indent=1)
    shutil.copy(os.path.join(ub, "ubench7.txt"), os.path.join(dst, "ubench7.txt"))
    print(json.dumps(kernels, indent=1))


if __name__ == "__main__":
    main()
