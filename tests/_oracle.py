"""ctypes access to the CPU oracle (oracle/liboracle.so) and the compiled
reference (oracle/_ref/pt_ref). TEST INFRASTRUCTURE: only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, and
only as the checker."""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
import tempfile
from typing import Optional, Sequence, Tuple

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.environ.get("PT_ORACLE_LIB") or os.path.join(ROOT, "oracle", "liboracle.so")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "pt_ref")

NODE_DTYPE = np.dtype([("lb", "<f4", 3), ("rt", "<f4", 3), ("left", "<i4"), ("right", "<i4"),
                       ("tri_start", "<i4"), ("tri_end", "<i4")])
assert NODE_DTYPE.itemsize == 40

_lib: Optional[C.CDLL] = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = C.CDLL(ORACLE_SO)
        P = C.c_void_p
        L.oracle_bvh_build.argtypes = [C.c_int, P, P, P]
        L.oracle_camera.argtypes = [P, P, P, C.c_int, C.c_int, C.c_float, C.c_float, P]
        L.oracle_render.argtypes = [C.c_int, P, P, P, C.c_int, P, P, P, C.c_int, C.c_int, C.c_uint32,
                                    C.c_int, C.c_int, P, P]
        L.oracle_render_pixels.argtypes = [C.c_int, P, P, P, C.c_int, P, P, P, C.c_int, C.c_int,
                                           C.c_uint32, P, C.c_int, P, P]
        L.oracle_sample_seed.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.oracle_sample_seed.restype = C.c_uint32
        L.oracle_lcg.argtypes = [C.c_uint32, C.c_int, P, P]
        L.oracle_acosf.argtypes = [C.c_float]
        L.oracle_acosf.restype = C.c_float
        L.oracle_acosf_n.argtypes = [P, C.c_int, P]
        L.oracle_sincosf_n.argtypes = [P, C.c_int, P, P]
        L.oracle_libm_sweep.argtypes = [C.c_int, C.c_float, C.c_float, P]
        L.oracle_libm_sweep.restype = C.c_uint64
        L.oracle_tri_hit.argtypes = [P, P, P, P]
        L.oracle_theta_grid_check.argtypes = [P]
        L.oracle_theta_grid_check.restype = C.c_uint64
        L.oracle_slab.argtypes = [P, P, P, P]
        L.oracle_brdf.argtypes = [C.c_uint32, C.c_int, C.c_float, P, P, P]
        L.oracle_brdf.restype = C.c_uint32
        L.oracle_last_stats.argtypes = [P]
        L.oracle_rgb8.argtypes = [P, C.c_int, C.c_int, C.c_float, P]
        L.oracle_rgb8_sweep.argtypes = [C.c_float, P, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int]
        L.oracle_rgb8_sweep.restype = C.c_uint64
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def pack_scene(scene) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """verts (n,9) f32, material type (n,) i32, material values (n,7) f32."""
    verts = np.array([[c for p in t for c in p] for t in scene.tris], dtype=np.float64).astype(np.float32)
    mtype = np.array([m.type for m in scene.mats], dtype=np.int32)
    mvals = np.array([[*m.color, *m.emit, m.roughness] for m in scene.mats], dtype=np.float64).astype(np.float32)
    return np.ascontiguousarray(verts), mtype, np.ascontiguousarray(mvals)


def bvh_build(verts: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    n = verts.shape[0]
    nodes = np.zeros(max(2 * n - 1, 1), dtype=NODE_DTYPE)
    idx = np.zeros(n, dtype=np.int32)
    cnt = lib().oracle_bvh_build(n, _p(verts), _p(nodes), _p(idx))
    return nodes[:cnt].copy(), idx


def camera(scene) -> np.ndarray:
    c = scene.camera
    out = np.zeros(18, dtype=np.float32)
    f = lambda v: np.array(v, dtype=np.float64).astype(np.float32)
    rc = lib().oracle_camera(_p(f(c.pos)), _p(f(c.forward)), _p(f(c.up)), c.res[0], c.res[1],
                             C.c_float(np.float32(c.fov)), C.c_float(np.float32(c.distance)), _p(out))
    if rc != 0:
        raise ValueError("up vector too close to forward vector")
    return out


def render(scene, spp: int, depth: int, seed: int = 1, rows: Optional[Tuple[int, int]] = None,
           nodes: Optional[np.ndarray] = None, idx: Optional[np.ndarray] = None):
    """Oracle render of rows [r0, r1) -> ((r1-r0), W, 3) float32 linear mean, rays."""
    verts, mtype, mvals = pack_scene(scene)
    if nodes is None:
        nodes, idx = bvh_build(verts)
    cam = camera(scene)
    W, H = scene.camera.res
    r0, r1 = rows if rows else (0, H)
    out = np.zeros((r1 - r0, W, 3), dtype=np.float32)
    rays = C.c_uint64(0)
    lib().oracle_render(verts.shape[0], _p(verts), _p(mtype), _p(mvals), nodes.shape[0], _p(nodes), _p(idx),
                        _p(cam), spp, depth, seed, r0, r1, _p(out), C.byref(rays))
    return out, rays.value


def last_stats() -> dict:
    """Counters of the last oracle render (SURVEY.md Appendix C quantities)."""
    a = np.zeros(4, dtype=np.uint64)
    lib().oracle_last_stats(_p(a))
    return dict(rays=int(a[0]), node_visits=int(a[1]), tri_tests=int(a[2]), hits=int(a[3]))


def render_pixels(scene, pixels: Sequence[Tuple[int, int]], spp: int, depth: int, seed: int = 1):
    verts, mtype, mvals = pack_scene(scene)
    nodes, idx = bvh_build(verts)
    cam = camera(scene)
    px = np.ascontiguousarray(np.array(pixels, dtype=np.int32).reshape(-1, 2))
    out = np.zeros((px.shape[0], 3), dtype=np.float32)
    rays = C.c_uint64(0)
    lib().oracle_render_pixels(verts.shape[0], _p(verts), _p(mtype), _p(mvals), nodes.shape[0], _p(nodes),
                               _p(idx), _p(cam), spp, depth, seed, _p(px), px.shape[0], _p(out), C.byref(rays))
    return out, rays.value


def rgb8(img: np.ndarray, gamma: float = 2.2) -> np.ndarray:
    """gamma_correct + save_png's bytes (image.h:41-55), top row first."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    H, W = img.shape[:2]
    out = np.empty((H, W, 3), dtype=np.uint8)
    lib().oracle_rgb8(_p(img), W, H, C.c_float(gamma), _p(out))
    return out


# ---------------------------------------------------------------- reference binary
def ref_available() -> bool:
    return os.access(REF_BIN, os.X_OK)


def ref_run(scene, spp: int, depth: int, seed: int = 1, rows=None, extra: Sequence[str] = (),
            pixels=None, timeout: float = 600):
    """Run the compiled reference (oracle/_ref/pt_ref); returns (array, meta)."""
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "s.ptscene")
        with open(sp, "w") as f:
            f.write(scene.to_ptscene())
        out = os.path.join(td, "out.f32")
        W, H = scene.camera.res
        cmd = [REF_BIN, "--scene", sp, "--spp", str(spp), "--depth", str(depth), "--seed", str(seed),
               "--out", out, *extra]
        if rows:
            cmd += ["--rows", str(rows[0]), str(rows[1])]
        if pixels is not None:
            pf = os.path.join(td, "px.txt")
            with open(pf, "w") as f:
                f.write("\n".join(f"{w} {h}" for w, h in pixels) + "\n")
            cmd += ["--pixels", pf]
        r = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout)
        meta = json.loads(r.stdout.strip().splitlines()[-1])
        arr = np.fromfile(out, dtype=np.float32)
        if pixels is not None:
            arr = arr.reshape(-1, 3)
        else:
            r0, r1 = rows if rows else (0, H)
            arr = arr.reshape(r1 - r0, W, 3)
        return arr, meta
