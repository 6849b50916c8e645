#!/usr/bin/env python3
"""Fixed per-launch cost of a rank's share: one part of the N-way row
partition rendered at several spp counts on this GPU (each one trace launch), kernel time
from HIP events. A fit kernel_ms = a * spp + t gives t, the launch's fixed tail (ramp-up,
drain, clocks); t / (a * spp) is the share's excess over ideal that no work split removes.

usage: python scripts/part_tail.py --scene sphere --res 1024 --depth 5 --part 0/8 --spp 500 1000 2000 4000
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", choices=["cornell", "sphere"], default="sphere")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--part", default="0/8")
    ap.add_argument("--band", type=int, default=1)
    ap.add_argument("--spp", type=int, nargs="+", default=[500, 1000, 2000, 4000])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="samples per launch (0: as the library picks)")
    a = ap.parse_args()
    import numpy as np
    import ptamd
    from ptamd import scenes
    sc = scenes.cornell((a.res, a.res)) if a.scene == "cornell" else scenes.sphere_in_cornell(223, (a.res, a.res))
    bvh = ptamd.BVH.from_scene(sc)
    bvh.build()
    cam = ptamd.Camera.from_spec(sc.camera)
    r = ptamd.Renderer(0)
    r.set_scene(bvh)
    r.prepare()
    pi, pc = (int(v) for v in a.part.split("/"))
    rows = []
    for spp in a.spp:
        r.render(cam, spp, a.depth, part_index=pi, part_count=pc, band_rows=a.band, batch_spp=a.batch)  # warm-up
        ks = []
        for _ in range(a.reps):
            _, st = r.render(cam, spp, a.depth, part_index=pi, part_count=pc, band_rows=a.band, batch_spp=a.batch)
            ks.append(st["kernel_ms"])
        rows.append({"spp": spp, "kernel_ms": ks, "trace_launches": st["trace_launches"], "rays": st["rays"]})
        print(f"spp {spp}: kernel {min(ks):.3f} ms ({st['trace_launches']} launches)", file=sys.stderr, flush=True)
    x = np.array([row["spp"] for row in rows], dtype=np.float64)
    y = np.array([min(row["kernel_ms"]) for row in rows])
    slope, t = np.polyfit(x, y, 1)
    print(json.dumps({"workload": f"{sc.name}_{a.res}_d{a.depth}_part{a.part}", "rows": rows, "ms_per_spp": slope,
                      "fixed_ms": t, "fixed_over_1000spp": t / (slope * 1000)}))
    r.close()


if __name__ == "__main__":
    main()
