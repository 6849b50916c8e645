#!/usr/bin/env python3
"""Config 4's VALU issue and lane utilisation by section, from the duplication PMC passes
(scripts/gpu_r05b.sh -> gpurun_out/pmcv_<tag>/): for each section s, the variant that runs s
twice minus the base build gives s's main-port slots per ray (SQ_ACTIVE_INST_VALU -
SQ_ACTIVE_INST_VALU2), its VALU instructions per ray, the share of the kernel's time it takes
(1 / rate difference), and its lane utilisation (delta SQ_THREAD_CYCLES_VALU / (64 x delta
SQ_ACTIVE_INST_VALU)).
Sections are the variant directories present under the tag (any subset of NAMES).
usage: python scripts/section_split.py TAG OUT_DIR"""
import collections
import csv
import glob
import json
import os
import sys

tag, dst = sys.argv[1], sys.argv[2]
src = f"gpurun_out/pmcv_{tag}"
NAMES = {"node": "node test (wide_node_test)", "tri": "drain triangle tests", "cam": "camera ray",
         "brdf": "hemisphere sample", "fold": "unwinding (run for every path)", "scan": "step popcount + prefix sum",
         "enq": "step enqueue loop", "stack": "step stack push / pop", "drainq": "drain queue read + owner fetch",
         "shade": "shade: hit record, material, face-forward, hit point",
         "offs": "node load offsets (wide_offsets)", "xbox": "exact leaf-box check of a hit",
         "loopctl": "step loop exit test", "start": "segment start: 1 / d, range checks",
         "claim": "work claim item arithmetic", "camf": "camera ray (flat kernel)",
         "mask": "leaf-box mask (box tests + ballot chain)", "pair": "pair-round triangle test"}


def counters(name):
    acc = collections.Counter()
    for f in glob.glob(f"{src}/{name}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "trace" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    b = json.loads(open(f"{src}/{name}.json").read().strip().splitlines()[-1])
    return acc, b["rays_per_step"], b["kernel_mrays"]


base, rays, rate0 = counters("base")
main0 = (base["SQ_ACTIVE_INST_VALU"] - base["SQ_ACTIVE_INST_VALU2"]) / rays
out = {"base": {"main_port_per_ray": round(main0, 3), "valu_per_ray": round(base["SQ_INSTS_VALU"] / rays, 3),
                "lanes": round(base["SQ_THREAD_CYCLES_VALU"] / base["SQ_ACTIVE_INST_VALU"] / 64, 3),
                "kernel_mrays": round(rate0)}, "sections": {}}
print(f"{'section':52s} {'main/ray':>8s} {'valu/ray':>8s} {'time %':>7s} {'lanes':>6s}")
tot = 0.0
present = [n for n in NAMES if os.path.exists(f"{src}/{n}.json")]
for n in present:
    label = NAMES[n]
    c, _, rate = counters(n)
    dm = ((c["SQ_ACTIVE_INST_VALU"] - c["SQ_ACTIVE_INST_VALU2"]) - (base["SQ_ACTIVE_INST_VALU"] - base["SQ_ACTIVE_INST_VALU2"])) / rays
    dv = (c["SQ_INSTS_VALU"] - base["SQ_INSTS_VALU"]) / rays
    dact = c["SQ_ACTIVE_INST_VALU"] - base["SQ_ACTIVE_INST_VALU"]
    lanes = (c["SQ_THREAD_CYCLES_VALU"] - base["SQ_THREAD_CYCLES_VALU"]) / dact / 64 if dact > 0 else float("nan")
    tshare = (1 / rate - 1 / rate0) * rate0
    out["sections"][n] = {"label": label, "main_port_per_ray": round(dm, 3), "valu_per_ray": round(dv, 3),
                          "time_share": round(tshare, 4), "lanes": round(lanes, 3), "kernel_mrays_dup": round(rate)}
    if n != "fold":
        tot += dm
    print(f"{label:52s} {dm:8.3f} {dv:8.3f} {100 * tshare:7.1f} {lanes:6.3f}")
out["rest_main_port_per_ray"] = round(main0 - tot, 3)
print(f"{'rest (sections not duplicated in this tag)':52s} {main0 - tot:8.3f}")
print(f"{'total (base)':52s} {main0:8.3f}  lanes {out['base']['lanes']}")
os.makedirs(dst, exist_ok=True)
json.dump(out, open(os.path.join(dst, "section_split.json"), "w"), indent=1)
