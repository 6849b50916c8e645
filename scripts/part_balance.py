#!/usr/bin/env python3
"""Per-rank share of the multi-GPU row partition, timed alone on one GPU.

For each N in --ns, every part P of the N-way partition (rows dealt in 8-row bands,
row h -> part (h / 8) % N: what rank P renders at --gpus N) is rendered on this GPU and
timed (trace-kernel time from HIP events, and the render call's wall time). The frame is
rendered whole too. Balance = slowest part / (whole frame / N): 1.0 is ideal strong
scaling before the gather. Optionally the whole frame once more through the in-process
multi-device path with the RCCL gather forced as send-to-self (PT_GATHER=rccl), for the
gather time of a full frame.

usage: python scripts/part_balance.py --scene cornell --res 4096 --spp 10000 --depth 8 \
           --ns 2 4 8 [--rccl] > out.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", choices=["cornell", "sphere"], default="cornell")
    ap.add_argument("--res", type=int, default=4096)
    ap.add_argument("--spp", type=int, default=10000)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--band", type=int, default=8)
    ap.add_argument("--ns", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=1, help="timed renders per part (after one warm-up)")
    ap.add_argument("--rccl", action="store_true", help="also the whole frame through PT_GATHER=rccl (send-to-self)")
    a = ap.parse_args()
    import ptamd
    from ptamd import scenes
    sc = scenes.cornell((a.res, a.res)) if a.scene == "cornell" else scenes.sphere_in_cornell(223, (a.res, a.res))
    bvh = ptamd.BVH.from_scene(sc)
    bvh.build()
    cam = ptamd.Camera.from_spec(sc.camera)
    r = ptamd.Renderer(0)
    r.set_scene(bvh)
    r.prepare()

    def timed(pi, pc):
        r.render(cam, a.spp, a.depth, part_index=pi, part_count=pc, band_rows=a.band)  # warm-up
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            _, st = r.render(cam, a.spp, a.depth, part_index=pi, part_count=pc, band_rows=a.band)
            wall = (time.perf_counter() - t0) * 1e3
            row = {"kernel_ms": st["kernel_ms"], "wall_ms": wall, "rays": st["rays"], "rows": st["rows"],
                   "kernel_path": st["kernel_path"]}
            best = row if best is None or row["wall_ms"] < best["wall_ms"] else best
        return best

    out = {"workload": f"{sc.name}_{a.res}x{a.res}_spp{a.spp}_depth{a.depth}", "band_rows": a.band}
    whole = timed(0, 1)
    out["whole"] = whole
    print(f"whole frame: {whole['wall_ms']:.1f} ms (kernel {whole['kernel_ms']:.1f} ms)", file=sys.stderr, flush=True)
    out["partitions"] = {}
    for n in a.ns:
        parts = []
        for p in range(n):
            t = timed(p, n)
            parts.append(t)
            print(f"N={n} part {p}: {t['wall_ms']:.1f} ms (kernel {t['kernel_ms']:.1f}), {t['rows']} rows",
                  file=sys.stderr, flush=True)
        worst = max(parts, key=lambda t: t["wall_ms"])
        ideal = whole["wall_ms"] / n
        out["partitions"][str(n)] = {
            "parts": parts, "worst_wall_ms": worst["wall_ms"], "ideal_wall_ms": ideal,
            "worst_over_ideal": worst["wall_ms"] / ideal,
            "worst_kernel_over_ideal": max(t["kernel_ms"] for t in parts) / (whole["kernel_ms"] / n),
            "rays_sum_equals_whole": sum(t["rays"] for t in parts) == whole["rays"]}
    r.close()
    if a.rccl:
        # the in-process multi-device path, one device, the gather forced through RCCL's
        # send-to-self: the full frame's bytes cross RCCL and the assembly kernel runs
        os.environ["PT_TEST_HOOKS"] = "1"
        os.environ["PT_GATHER"] = "rccl"
        t0 = time.perf_counter()
        img, st = ptamd.render(cam, bvh, a.spp, a.depth, devices=[0])
        out["rccl_send_to_self"] = {"gather_path": ptamd._lib.pt_stats.GATHERS.get(st["gather_path"]),
                                    "gather_ms": st["gather_ms"], "total_ms": st["total_ms"],
                                    "wall_ms": (time.perf_counter() - t0) * 1e3,
                                    "frame_bytes": int(img.nbytes), "rays": st["rays"]}
        print(f"rccl send-to-self: gather {st['gather_ms']:.2f} ms, path {out['rccl_send_to_self']['gather_path']}",
              file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
