#!/usr/bin/env python3
"""Summarise the round-5 VALU issue microbenchmark (scripts/gpu_r05_ubench.sh) into
profiles/<tag>/valu_peak.json and a table: cycles per wave64 instruction per SIMD for
v_fma_f32, v_pk_fma_f32, v_add_f32, v_max3_f32 (+ v_mul_f32, fma+add alternating) at 1, 2,
4 and 8 waves per SIMD, the second-port share (SQ_ACTIVE_INST_VALU2 / SQ_ACTIVE_INST_VALU,
1 and 8 waves), and the FP32 rate each implies over 256 CUs x 4 SIMDs at 2.4 GHz against
MI355X_MICROARCH.md's 157.3 TFLOP/s vector spec (its rows 54 and 473: "v_fma_f32 (wave64)
2 cyc (SIMD-32); one wave alone: 4").
usage: python scripts/valu_peak.py gpurun_out/r05_ubench TAG"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLOPS = {"fma": 2, "pk_fma": 4, "add": 1, "mul": 1, "fma+add": 1.5, "max3": 0}  # per lane per instruction
SPEC_TF = 157.3


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out = {"ubench": "tools/valu_ubench: 8 independent dependency chains per wave, 4096 x 8 instructions per "
                     "wave, a full grid of 256-thread blocks (waves per SIMD as listed)", "spec_fp32_tflops": SPEC_TF,
           "forms": collections.OrderedDict()}
    for w in (1, 2, 4, 8):
        p = os.path.join(src, f"ubench_w{w}.txt")
        if not os.path.exists(p):
            continue
        for line in open(p):
            m = re.match(r"(\S+)\s+([\d.]+) cycles per wave-instruction per SIMD", line)
            if not m:
                continue
            name, cyc = m.group(1), float(m.group(2))
            f = out["forms"].setdefault(name, {"cycles_per_inst": {}, "tflops_implied": {}, "second_port_share": {}})
            f["cycles_per_inst"][w] = cyc
            if FLOPS.get(name):
                f["tflops_implied"][w] = round(FLOPS[name] * 64 / cyc * 2.4e9 * 1024 / 1e12, 1)
    for w in (1, 8):
        acc = collections.defaultdict(collections.Counter)
        for p in glob.glob(os.path.join(src, f"pmc_w{w}", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
        # kernels are ubench<op>; op numbers in tools/valu_ubench.hip's table order
        ops = {0: "fma", 1: "pk_fma", 9: "add", 8: "max3", 18: "mul", 26: "fma+add"}
        for k, c in acc.items():
            m = re.search(r"<(\d+)>", k)
            if not m or int(m.group(1)) not in ops or not c["SQ_ACTIVE_INST_VALU"]:
                continue
            name = ops[int(m.group(1))]
            if name in out["forms"]:
                out["forms"][name]["second_port_share"][w] = round(c["SQ_ACTIVE_INST_VALU2"] / c["SQ_ACTIVE_INST_VALU"], 3)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    json.dump(out, open(os.path.join(dst, "valu_peak.json"), "w"), indent=1)
    ws = (1, 2, 4, 8)
    print("| form | " + " | ".join(f"cycles @{w} w/SIMD" for w in ws) + " | TFLOP/s implied @8 | 2nd port @1 / @8 |")
    print("|---|" + "---|" * (len(ws) + 2))
    for name, f in out["forms"].items():
        cyc = " | ".join(f"{f['cycles_per_inst'].get(w, float('nan')):.2f}" for w in ws)
        tf = f["tflops_implied"].get(8, "—")
        sp = f"{f['second_port_share'].get(1, '—')} / {f['second_port_share'].get(8, '—')}"
        print(f"| {name} | {cyc} | {tf} | {sp} |")


if __name__ == "__main__":
    main()
