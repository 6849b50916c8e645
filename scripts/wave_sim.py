#!/usr/bin/env python3
"""Wave-level statistics of the flat kernel's work, from a statistical CPU path tracer
(numpy; the reference's scene, camera, BRDFs and depth, NOT bit-exact — an estimate of how
rays fall into waves, for design questions that depend on it).

A wave holds 64 paths; a lane whose path ends takes the next work item (consecutive pixels
of one sample, as `pt_trace.h` refills: item = sample block * npix + pixel), so at every
wave-iteration the lanes trace one segment each of paths at mixed depths. Two questions:

1. Two-level box mask: with leaf groups = the BVH's subtrees at depth 1
   and 2, how often do ALL active lanes of a wave miss a group's box (the only case in
   which a wave-uniform group test lets the wave skip that group's leaf tests)?
2. Specular rejection loop (`material.h:20-23`): lanes shading a SPECULAR hit loop until a
   jittered reflection leaves the surface; a wave pays max-over-lanes trips. Mean trips per
   specular lane against the wave's max.

usage: python scripts/wave_sim.py [--scene cornell|mcornell] [--rough R] [--paths N]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))



def load(scene, rough):
    import ptamd
    from ptamd import scenes
    global EMIT, DIFFUSE, SPECULAR
    EMIT, DIFFUSE, SPECULAR = scenes.EMIT, scenes.DIFFUSE, scenes.SPECULAR
    sc = scenes.cornell((1024, 1024)) if scene == "cornell" else scenes.modified_cornell(rough, (1024, 1024))
    tris = np.array([[list(v) for v in t] for t in sc.tris], dtype=np.float64)
    mtype = np.array([m.type for m in sc.mats])
    rgh = np.array([m.roughness for m in sc.mats], dtype=np.float64)
    bvh = ptamd.BVH.from_scene(sc)
    bvh.build()
    return sc, tris, mtype, rgh, bvh.nodes, bvh.tri_idx


def intersect(tris, o, d):
    """nearest hit (t > 1e-7 relative guard), Moller-Trumbore over all triangles."""
    v0, e1, e2 = tris[:, 0], tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0]
    p = np.cross(d[:, None, :], e2[None])
    det = np.einsum("nti,ti->nt", p, e1)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / det
        s = o[:, None, :] - v0[None]
        u = np.einsum("nti,nti->nt", s, p) * inv
        q = np.cross(s, e1[None])
        v = np.einsum("ni,nti->nt", d, q) * inv
        t = np.einsum("ti,nti->nt", e2, q) * inv
    ok = (np.abs(det) > 1e-12) & (u >= 0) & (v >= 0) & (u + v <= 1) & (t > 1e-6)
    t = np.where(ok, t, np.inf)
    hit = np.argmin(t, axis=1)
    tt = t[np.arange(len(t)), hit]
    return np.where(np.isfinite(tt), hit, -1), tt


def trace_paths(sc, tris, mtype, rgh, n, depth, rng):
    """n paths in work-item order (consecutive pixels, sample 0): per path its segments'
    (o, d) and, per segment that shades a SPECULAR hit, the rejection loop's trips."""
    W, H = sc.camera.res
    pos = np.array(sc.camera.pos)
    F = np.array(sc.camera.forward, dtype=np.float64)
    F /= np.linalg.norm(F)
    R = np.cross(sc.camera.forward, sc.camera.up)
    R /= np.linalg.norm(R)
    U = np.cross(R, F)
    vx = 2 * np.tan(np.radians(sc.camera.fov) / 2)
    vy = vx * H / W
    start = rng.integers(0, W * H - n) if n < W * H else 0
    q = start + np.arange(n)
    x, y = q % W + rng.random(n), q // W + rng.random(n)
    d = F[None] + ((x / W - 0.5) * vx)[:, None] * R[None] + ((0.5 - y / H) * vy)[:, None] * U[None]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.repeat(pos[None], n, axis=0)
    segs = [[] for _ in range(n)]
    trips = [[] for _ in range(n)]
    live = np.arange(n)
    for k in range(depth):
        if not len(live):
            break
        for i, oo, dd in zip(live, o, d):
            segs[i].append((oo, dd))
        hit, t = intersect(tris, o, d)
        keep = hit >= 0
        if k + 1 < depth:
            keep &= mtype[np.maximum(hit, 0)] != EMIT
        else:
            keep[:] = False
        live, o, d, hit, t = live[keep], o[keep], d[keep], hit[keep], t[keep]
        if not len(live):
            break
        e1, e2 = tris[hit, 1] - tris[hit, 0], tris[hit, 2] - tris[hit, 0]
        nrm = np.cross(e1, e2)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        nrm = np.where((np.einsum("ni,ni->n", nrm, d) < 0)[:, None], nrm, -nrm)
        p = o + d * t[:, None]
        nd = np.empty_like(d)
        spec = mtype[hit] == SPECULAR
        # diffuse: uniform hemisphere (theta = acos(2u-1) - pi/2, phi = 2 pi v, flipped)
        dm = ~spec
        if dm.any():
            u, v = rng.random(dm.sum()), rng.random(dm.sum())
            th, ph = np.arccos(2 * u - 1) - np.pi / 2, 2 * np.pi * v
            s = np.stack([np.cos(th) * np.cos(ph), np.cos(th) * np.sin(ph), np.sin(th)], 1)
            flip = np.einsum("ni,ni->n", s, nrm[dm]) < 0
            nd[dm] = np.where(flip[:, None], -s, s)
        if spec.any():
            idx = np.nonzero(spec)[0]
            refl = d[idx] - 2 * np.einsum("ni,ni->n", d[idx], nrm[idx])[:, None] * nrm[idx]
            r = rgh[hit[idx]]
            cnt = np.zeros(len(idx), dtype=np.int64)
            out = np.zeros((len(idx), 3))
            todo = np.arange(len(idx))
            while len(todo):
                cnt[todo] += 1
                j = (rng.random((len(todo), 3)) - 0.5) * r[todo, None]
                c = refl[todo] + j
                ok = np.einsum("ni,ni->n", c, nrm[idx[todo]]) >= 0
                out[todo[ok]] = c[ok]
                todo = todo[~ok]
            nd[idx] = out / np.linalg.norm(out, axis=1, keepdims=True)
            for ii, c in zip(live[idx], cnt):
                trips[ii].append((len(segs[ii]) - 1, int(c)))
        o, d = p + nrm * 1e-4, nd
    return segs, trips


def subtree_groups(nodes, level):
    """(leaf-rank ranges are not needed here): the boxes of the BVH's nodes at `level`."""
    out, frontier = [], [0]
    for _ in range(level):
        nxt = []
        for i in frontier:
            if nodes[i]["left"] >= 0 and nodes[i]["right"] >= 0:
                nxt += [int(nodes[i]["left"]), int(nodes[i]["right"])]
            else:
                nxt.append(i)
        frontier = nxt
    return [(np.array(nodes[i]["lb"], dtype=np.float64), np.array(nodes[i]["rt"], dtype=np.float64)) for i in frontier]


def passes(lb, rt, o, d):
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t1, t2 = (lb[None] - o) * inv, (rt[None] - o) * inv
    t1, t2 = np.nan_to_num(t1, nan=-np.inf), np.nan_to_num(t2, nan=np.inf)
    tmin = np.maximum(np.max(np.minimum(t1, t2), axis=1), 0.0)
    tmax = np.min(np.maximum(t1, t2), axis=1)
    return tmin <= tmax


def simulate(segs, trips, lanes=64):
    """wave-iterations: each lane traces its path's next segment; an ended path's lane takes
    the next path (work item). Returns per iteration the (o, d) of the active lanes and the
    specular trips of lanes shading specular hits."""
    nxt, cur, pos = 0, [-1] * lanes, [0] * lanes
    tripmap = [dict(t) for t in trips]
    its = []
    while True:
        for l in range(lanes):
            if cur[l] < 0 or pos[l] >= len(segs[cur[l]]):
                if nxt < len(segs):
                    cur[l], pos[l] = nxt, 0
                    nxt += 1
                else:
                    cur[l] = -2
        act = [l for l in range(lanes) if cur[l] >= 0]
        if not act:
            break
        od = [segs[cur[l]][pos[l]] for l in act]
        tr = [tripmap[cur[l]].get(pos[l]) for l in act]
        its.append((np.array([a for a, _ in od]), np.array([b for _, b in od]), [t for t in tr if t]))
        for l in act:
            pos[l] += 1
        if nxt >= len(segs) and len(act) < lanes // 2:
            break  # drain tail: not the steady state
    return its


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", choices=["cornell", "mcornell"], default="cornell")
    ap.add_argument("--rough", type=float, default=0.8)
    ap.add_argument("--paths", type=int, default=20000)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    sc, tris, mtype, rgh, nodes, _ = load(a.scene, a.rough)
    segs, trips = trace_paths(sc, tris, mtype, rgh, a.paths, a.depth, rng)
    its = simulate(segs, trips)
    nseg = sum(len(s) for s in segs)
    out = {"scene": sc.name, "paths": a.paths, "segments": nseg, "segments_per_path": nseg / a.paths,
           "wave_iterations": len(its)}
    for level in (1, 2):
        groups = subtree_groups(nodes, level)
        skip = []
        lane_pass = []
        for lb, rt in groups:
            hits = [passes(lb, rt, o, d) for o, d, _ in its]
            skip.append(float(np.mean([not h.any() for h in hits])))
            lane_pass.append(float(np.mean(np.concatenate(hits))))
        out[f"groups_level{level}"] = {"count": len(groups), "lane_pass_rate": lane_pass,
                                       "wave_skip_rate": skip}
    spec_lanes = [t for _, _, tr in its for t in tr]
    if spec_lanes:
        waves = [tr for _, _, tr in its if tr]
        out["specular"] = {
            "lanes_per_iteration_with_specular": float(np.mean([len(t) for t in waves])),
            "iterations_with_specular_frac": len(waves) / len(its),
            "mean_trips_per_lane": float(np.mean(spec_lanes)),
            "mean_max_trips_per_wave": float(np.mean([max(t) for t in waves])),
            "trip_histogram": np.bincount(np.array(spec_lanes), minlength=8)[:12].tolist(),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
