"""ptamd — Python host layer over libpt_hip.so, mirroring the reference's C++ API.

Reference interface (Blackgaurd/pathtracer-cpp, pathtracer/):
  Material(type, color, emit_color, roughness)     material.h:27-52
  Triangle(v1, v2, v3, material)                   triangle.h:7-23
  BVH.add_triangle / size / empty / build          bvh.h:30-155
  Camera(pos, forward, up, res, fov, distance)     camera.h:33-61
  render_cpu(camera, bvh, samples, depth, file)    render.h:62-104
  render_gpu(camera, bvh, samples, depth, chunk, file) render.h:109-152

Both render entry points run the gfx950 trace kernel (the reference's CPU loop
and its GL tile loop are the path being replaced); they keep the reference's
argument meaning, messages and bool/exception behaviour. `render()` returns the
linear image (the mean after /spp, before gamma) for programmatic use.
"""
from __future__ import annotations

import array
import ctypes as C
import itertools
import math
import operator
import os
import sys
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import PT_MAX_DEPTH, PT_SEED, PTError, build, check, lib  # noqa: F401
from . import scenes  # noqa: F401

EMIT, DIFFUSE, SPECULAR = 1, 2, 3

NODE_DTYPE = np.dtype([("lb", "<f4", 3), ("rt", "<f4", 3), ("left", "<i4"), ("right", "<i4"),
                       ("tri_start", "<i4"), ("tri_end", "<i4")])
# pt_material (include/pt_hip.h, material.h:27-37): 32 bytes, no padding
MATERIAL_DTYPE = np.dtype([("type", "<i4"), ("color", "<f4", 3), ("emit", "<f4", 3), ("roughness", "<f4")])
assert MATERIAL_DTYPE.itemsize == C.sizeof(_lib.pt_material)


def _f3(v) -> Tuple[float, float, float]:
    if isinstance(v, (int, float)):
        return (float(v),) * 3
    return tuple(float(c) for c in v)


@dataclass
class Material:
    type: int
    color: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    emit_color: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    roughness: float = 0.0
    EMIT = EMIT
    DIFFUSE = DIFFUSE
    SPECULAR = SPECULAR

    def __post_init__(self):
        self.color = _f3(self.color)
        self.emit_color = _f3(self.emit_color)
        self.roughness = float(self.roughness)


@dataclass
class Triangle:
    v1: Tuple[float, float, float]
    v2: Tuple[float, float, float]
    v3: Tuple[float, float, float]
    material: Material


@dataclass
class BVH:
    """Scene container = the reference's BVH (bvh.h:30-37): triangles + built tree."""
    triangles: List[Triangle] = field(default_factory=list)
    built: bool = False
    nodes: Optional[np.ndarray] = None
    tri_idx: Optional[np.ndarray] = None

    def add_triangle(self, tri: Triangle) -> None:
        self.built = False
        self._packed = None
        self.triangles.append(tri)
        # the C ABI's fields appended as the triangle is added (the reference's Triangle
        # constructor works at add time too, triangle.h:14-23): build() and the scene upload
        # then view these buffers instead of converting ~10^5 Python objects (config 4: the
        # Python packing took longer than the builder itself)
        if self._inc is None:
            self._inc = (array.array("d"), array.array("d"), array.array("i"), [])
        vb, mb, tb, objs = self._inc
        if len(objs) == len(self.triangles) - 1:
            m = tri.material
            vb.extend(tri.v1)
            vb.extend(tri.v2)
            vb.extend(tri.v3)
            mb.extend(m.color)
            mb.extend(m.emit_color)
            mb.append(m.roughness)
            tb.append(m.type)
            objs.append(tri)

    def size(self) -> int:
        return len(self.triangles)

    def empty(self) -> bool:
        return not self.triangles

    # packed arrays in the C ABI layout, made once per triangle list (build() and every
    # renderer's scene upload share them; add_triangle drops them)
    _packed: Optional[tuple] = field(default=None, init=False, repr=False, compare=False)
    # add_triangle's buffers: (vertices as doubles, color / emit / roughness as doubles,
    # material types, the triangles they were taken from)
    _inc: Optional[tuple] = field(default=None, init=False, repr=False, compare=False)

    def _pack(self) -> tuple:
        if self._packed is None or self._packed[0] != len(self.triangles):
            inc = self._inc
            if inc is not None and len(inc[3]) == len(self.triangles) and \
                    all(map(operator.is_, inc[3], self.triangles)):  # nothing replaced behind add_triangle
                self._packed = (len(self.triangles), self._verts_inc(), self._materials_inc())
            else:
                self._packed = (len(self.triangles), self._verts(), self._materials())
        return self._packed

    def _verts_inc(self) -> np.ndarray:
        v = np.frombuffer(self._inc[0], dtype=np.float64)
        return np.ascontiguousarray(v.astype(np.float32).reshape(-1, 9))

    def _materials_inc(self):
        n = len(self.triangles)
        vals = np.frombuffer(self._inc[1], dtype=np.float64).reshape(n, 7).astype(np.float32)
        arr = np.zeros(max(n, 1), dtype=MATERIAL_DTYPE)
        if n:
            arr["type"] = np.frombuffer(self._inc[2], dtype=np.int32)
            arr["color"] = vals[:, 0:3]
            arr["emit"] = vals[:, 3:6]
            arr["roughness"] = vals[:, 6]
        m = (_lib.pt_material * max(n, 1)).from_buffer(arr)
        m._keep = arr
        return m

    def verts(self) -> np.ndarray:
        return self._pack()[1]

    def materials(self):
        return self._pack()[2]

    def _verts(self) -> np.ndarray:
        # doubles rounded to float once, as the reference's vec3 constructor does
        n = len(self.triangles)
        v = np.fromiter(itertools.chain.from_iterable((*t.v1, *t.v2, *t.v3) for t in self.triangles),
                        dtype=np.float64, count=9 * n)
        return np.ascontiguousarray(v.astype(np.float32).reshape(-1, 9))

    def _materials(self):
        """pt_material per triangle: a ctypes array over a numpy buffer, filled column by
        column (each float rounded once to float32, as the reference's fields hold it)."""
        n = len(self.triangles)
        ms = [t.material for t in self.triangles]
        vals = np.fromiter(itertools.chain.from_iterable((*m.color, *m.emit_color, m.roughness) for m in ms),
                           dtype=np.float64, count=7 * n).reshape(n, 7).astype(np.float32)
        arr = np.zeros(max(n, 1), dtype=MATERIAL_DTYPE)
        if n:
            arr["type"] = np.fromiter((m.type for m in ms), dtype=np.int32, count=n)
            arr["color"] = vals[:, 0:3]
            arr["emit"] = vals[:, 3:6]
            arr["roughness"] = vals[:, 6]
        m = (_lib.pt_material * max(n, 1)).from_buffer(arr)
        m._keep = arr  # the ctypes array views arr's memory
        return m

    def build(self) -> None:
        """BVH::build (bvh.h:79-155), bit-identical output, O(n log^2 n)."""
        if self.built:
            return
        n = len(self.triangles)
        if n == 0:
            raise PTError(_lib.PT_E_EMPTY, "No triangles in scene.")
        verts = self.verts()
        nodes = np.zeros(2 * n - 1, dtype=NODE_DTYPE)
        idx = np.zeros(n, dtype=np.int32)
        cnt = check(lib().pt_bvh_build(n, verts.ctypes.data, nodes.ctypes.data, idx.ctypes.data))
        self.nodes, self.tri_idx, self.built = nodes[:cnt].copy(), idx, True

    def load_obj(self, filename: str, mtl_path: str = "./") -> None:
        """BVH::load_obj (bvh.h:184-242): the OBJ's triangles (tinyobjloader's parsing and
        triangulation, restated in csrc/pt_obj.cpp) with the bvh.h:220-238 material
        mapping, appended in file order. Raises PTError where the reference throws
        (unreadable file, malformed face) and where it has undefined behaviour (a face
        without a material, a vertex index past the end)."""
        h = C.c_void_p()
        check(lib().pt_obj_load(filename.encode(), mtl_path.encode(), C.byref(h)))
        try:
            warn = lib().pt_obj_warnings(h).decode(errors="replace")
            n = lib().pt_obj_num_tris(h)
            verts = np.empty((n, 9), dtype=np.float32)
            mats = (_lib.pt_material * max(n, 1))()
            illum = np.empty(n, dtype=np.int32)
            check(lib().pt_obj_triangles(h, verts.ctypes.data, C.addressof(mats), illum.ctypes.data))
        finally:
            lib().pt_obj_free(h)
        if warn:
            print("TinyObjLoader: " + warn, file=sys.stderr)
        v = verts.astype(np.float64).tolist()
        for i in range(n):
            if illum[i] not in (1, 2):
                print(f"Unknown material type with illum: {illum[i]}\nUsing default material: Diffuse(0.5)",
                      file=sys.stderr)
            m = mats[i]
            self.add_triangle(Triangle(tuple(v[i][0:3]), tuple(v[i][3:6]), tuple(v[i][6:9]),
                                       Material(m.type, tuple(m.color), tuple(m.emit), m.roughness)))

    @classmethod
    def from_scene(cls, scene) -> "BVH":
        b = cls()
        for (a, bb, c), m in zip(scene.tris, scene.mats):
            b.add_triangle(Triangle(a, bb, c, Material(m.type, m.color, m.emit, m.roughness)))
        return b


class Camera:
    """Camera ctor arithmetic (camera.h:33-61) computed by pt_camera_init."""

    def __init__(self, pos, forward, up, res: Tuple[int, int], fov: float, distance: float = 1.0):
        self.pos, self.forward, self.up = _f3(pos), _f3(forward), _f3(up)
        self.res = (int(res[0]), int(res[1]))
        self.fov = float(np.float32(fov))
        self.distance = float(np.float32(distance))
        self.c = _lib.pt_camera()
        f = lambda v: np.array(v, dtype=np.float64).astype(np.float32)
        p, fw, u = f(self.pos), f(self.forward), f(self.up)
        check(lib().pt_camera_init(p.ctypes.data, fw.ctypes.data, u.ctypes.data, self.res[0], self.res[1],
                                   C.c_float(self.fov), C.c_float(self.distance), C.byref(self.c)))

    @classmethod
    def from_spec(cls, spec) -> "Camera":
        return cls(spec.pos, spec.forward, spec.up, spec.res, spec.fov, spec.distance)


class _SceneRef:
    """Keeps the numpy/ctypes arrays alive while a pt_scene points into them."""

    def __init__(self, bvh: BVH):
        if bvh.empty():
            raise PTError(_lib.PT_E_EMPTY, "No triangles in scene.")
        if not bvh.built:
            bvh.build()
        self.verts = bvh.verts()
        self.mats = bvh.materials()
        self.nodes = np.ascontiguousarray(bvh.nodes)
        self.idx = np.ascontiguousarray(bvh.tri_idx, dtype=np.int32)
        self.s = _lib.pt_scene(len(bvh.triangles), self.verts.ctypes.data, C.addressof(self.mats),
                               self.nodes.shape[0], self.nodes.ctypes.data, self.idx.ctypes.data)


SCENE_INFO_KEYS = ("nodes", "tree_depth", "flat_leaves", "ref_stack", "wide_nodes", "wide_width", "wide_levels",
                   "wide_top", "wide_tris", "wide_record_bytes")


def scene_info(bvh: BVH) -> dict:
    """How the kernels will traverse `bvh` (pt_scene_info; no device needed)."""
    ref = _SceneRef(bvh)
    info = np.zeros(len(SCENE_INFO_KEYS), dtype=np.int32)
    check(lib().pt_scene_info(C.byref(ref.s), info.ctypes.data, len(info)))
    return dict(zip(SCENE_INFO_KEYS, info.tolist()))


class Renderer:
    """A device context (pt_ctx): scene resident in HBM, repeated renders."""

    def __init__(self, device: int = 0):
        self.device = device
        h = C.c_void_p()
        check(lib().pt_ctx_create(device, C.byref(h)))
        self.h = h

    def close(self) -> None:
        if getattr(self, "h", None):
            lib().pt_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def flags(self) -> dict:
        """How this context renders its scene (test hook pt_debug_ctx_flags)."""
        out = (C.c_int32 * 5)()
        check(lib().pt_debug_ctx_flags(self.h, out))
        return {"albedo_x2": bool(out[0]), "specular": bool(out[1]), "rtc": bool(out[2]), "wide_nodes": out[3],
                "dark": bool(out[4])}

    def set_scene(self, bvh: BVH) -> None:
        ref = _SceneRef(bvh)
        check(lib().pt_ctx_set_scene(self.h, C.byref(ref.s)))

    def prepare(self) -> None:
        """Wait for the scene's background hipRTC compile (pt_ctx_prepare)."""
        check(lib().pt_ctx_prepare(self.h))

    @staticmethod
    def part_rows(res_y: int, part_index: int, part_count: int, band_rows: int) -> int:
        return lib().pt_part_rows(res_y, part_index, part_count, band_rows)

    def render(self, camera: Camera, samples: int, depth: int, seed: int = PT_SEED, part_index: int = 0,
               part_count: int = 1, band_rows: int = 1, out=None, batch_spp: int = 0,
               samples_per_item: int = 0):
        """Render this part's rows. `out`: None (returns numpy), or a torch CUDA tensor
        (float32, rows*W*3 elements) written in place on this context's device."""
        W, H = camera.res
        rows = self.part_rows(H, part_index, part_count, band_rows)
        prm = _lib.pt_params(samples, depth, seed, part_index, part_count, band_rows, batch_spp, samples_per_item)
        st = _lib.pt_stats()
        if out is None:
            img = np.empty((rows, W, 3), dtype=np.float32)
            check(lib().pt_ctx_render(self.h, C.byref(camera.c), C.byref(prm), img.ctypes.data, 0, C.byref(st)))
            return img, st.as_dict()
        if out.numel() != rows * W * 3 or not out.is_contiguous():
            raise ValueError("out must be a contiguous tensor with rows*W*3 elements")
        check(lib().pt_ctx_render(self.h, C.byref(camera.c), C.byref(prm), C.c_void_p(out.data_ptr()), 1,
                                  C.byref(st)))
        return out, st.as_dict()

    def render_progressive(self, camera: Camera, s_first: int, s_count: int, depth: int, seed: int = PT_SEED,
                           part_index: int = 0, part_count: int = 1, band_rows: int = 1, out=None,
                           batch_spp: int = 0, samples_per_item: int = 0):
        """Frame accumulation (render_realtime, render.h:219-387, offscreen): adds samples
        [s_first, s_first + s_count) to this context's running sum and returns the running
        mean, bit-identical to render() with s_first + s_count samples. s_first = 0 starts
        a new sum; otherwise it must continue the last one (same camera, depth, seed and
        partition) or PTError is raised. Any other render on this context ends the sum."""
        W, H = camera.res
        rows = self.part_rows(H, part_index, part_count, band_rows)
        prm = _lib.pt_params(s_first + s_count, depth, seed, part_index, part_count, band_rows, batch_spp,
                             samples_per_item)
        st = _lib.pt_stats()
        if out is None:
            img = np.empty((rows, W, 3), dtype=np.float32)
            check(lib().pt_ctx_render_progressive(self.h, C.byref(camera.c), C.byref(prm), s_first, s_count,
                                                  img.ctypes.data, 0, C.byref(st)))
            return img, st.as_dict()
        if out.numel() != rows * W * 3 or not out.is_contiguous():
            raise ValueError("out must be a contiguous tensor with rows*W*3 elements")
        check(lib().pt_ctx_render_progressive(self.h, C.byref(camera.c), C.byref(prm), s_first, s_count,
                                              C.c_void_p(out.data_ptr()), 1, C.byref(st)))
        return out, st.as_dict()

    def render_rgb8(self, camera: Camera, samples: int, depth: int, gamma: float = 2.2, flip: bool = True,
                    seed: int = PT_SEED, part_index: int = 0, part_count: int = 1, band_rows: int = 1, out=None,
                    batch_spp: int = 0, samples_per_item: int = 0):
        """render() + gamma_correct + save_png quantisation on the device (render.h:97-100,
        image.h:41-55): uint8 (rows, W, 3), equal to to_rgb8(render(...)) for a whole image
        (flip=True: top row first). `out`: None (numpy) or a torch uint8 CUDA tensor."""
        W, H = camera.res
        rows = self.part_rows(H, part_index, part_count, band_rows)
        prm = _lib.pt_params(samples, depth, seed, part_index, part_count, band_rows, batch_spp, samples_per_item)
        st = _lib.pt_stats()
        if out is None:
            img = np.empty((rows, W, 3), dtype=np.uint8)
            check(lib().pt_ctx_render_rgb8(self.h, C.byref(camera.c), C.byref(prm), C.c_float(gamma), int(flip),
                                           img.ctypes.data, 0, C.byref(st)))
            return img, st.as_dict()
        if out.numel() != rows * W * 3 or not out.is_contiguous():
            raise ValueError("out must be a contiguous tensor with rows*W*3 elements")
        check(lib().pt_ctx_render_rgb8(self.h, C.byref(camera.c), C.byref(prm), C.c_float(gamma), int(flip),
                                       C.c_void_p(out.data_ptr()), 1, C.byref(st)))
        return out, st.as_dict()


def render(camera: Camera, bvh: BVH, samples: int, depth: int, seed: int = PT_SEED, device: int = 0,
           devices: Optional[Sequence[int]] = None, band_rows: int = 1, **kw):
    """Linear image (H, W, 3) float32, h = 0 the bottom row (Image::pixels), + stats.
    `devices`: render on several GPUs of this process (pt_render_f32_devices: row bands
    dealt to the devices, one host thread each); the image does not depend on it."""
    if devices is not None:
        if not bvh.built:
            bvh.build()
        ref = _SceneRef(bvh)
        W, H = camera.res
        dv = np.ascontiguousarray(devices, dtype=np.int32)
        prm = _lib.pt_params(samples, depth, seed, 0, len(dv), band_rows, kw.get("batch_spp", 0),
                             kw.get("samples_per_item", 0))
        img = np.empty((H, W, 3), dtype=np.float32)
        st = _lib.pt_stats()
        check(lib().pt_render_f32_devices(C.byref(ref.s), C.byref(camera.c), C.byref(prm), dv.ctypes.data,
                                          len(dv), img.ctypes.data, C.byref(st)))
        return img, st.as_dict()
    r = Renderer(device)
    try:
        r.set_scene(bvh)
        return r.render(camera, samples, depth, seed=seed, **kw)
    finally:
        r.close()


PROGRESS_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int64, C.c_int64)


def render_rgb8(camera: Camera, bvh: BVH, samples: int, depth: int, devices: Sequence[int], gamma: float = 2.2,
                seed: int = PT_SEED, band_rows: int = 1, progress=None, **kw):
    """render() on several GPUs of this process + gamma_correct / save_png quantisation on
    the first device after the RCCL gather (pt_render_rgb8_devices): (H, W, 3) uint8, top
    row first (the PNG's rows), + stats. progress(done, total): called as pixel-samples
    complete (pt_params.progress)."""
    if not bvh.built:
        bvh.build()
    ref = _SceneRef(bvh)
    W, H = camera.res
    dv = np.ascontiguousarray(devices, dtype=np.int32)
    prm = _lib.pt_params(samples, depth, seed, 0, len(dv), band_rows, kw.get("batch_spp", 0),
                         kw.get("samples_per_item", 0))
    cb = None
    if progress is not None:
        cb = PROGRESS_FN(lambda _user, done, total: progress(done, total))
        prm.progress = C.cast(cb, C.c_void_p)
    img = np.empty((H, W, 3), dtype=np.uint8)
    st = _lib.pt_stats()
    check(lib().pt_render_rgb8_devices(C.byref(ref.s), C.byref(camera.c), C.byref(prm), dv.ctypes.data, len(dv),
                                       C.c_float(gamma), img.ctypes.data, C.byref(st)))
    del cb
    return img, st.as_dict()


def devices_release() -> None:
    """Free the contexts pt_render_*_devices keeps per device list (pt_devices_release)."""
    lib().pt_devices_release()


def debug_counter(which: int) -> int:
    """Process-wide counters (test hook pt_debug_counter): 0 contexts created, 1 scene
    uploads, 2 cached device sets live, 3 uploads skipped on a cached context."""
    return int(lib().pt_debug_counter(which))


def visible_devices() -> List[int]:
    """Every visible GPU, or PT_DEVICES="0,2,..." (as the C++ drop-in)."""
    env = os.environ.get("PT_DEVICES", "")
    devs = [int(t) for t in env.split(",") if t.strip()]
    return devs or list(range(max(lib().pt_device_count(), 1)))


def to_rgb8(img: np.ndarray, gamma: float = 2.2) -> np.ndarray:
    """gamma_correct + save_png quantisation + flip (image.h:41-55): top row first."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    H, W = img.shape[:2]
    out = np.empty((H, W, 3), dtype=np.uint8)
    check(lib().pt_image_to_rgb8(img.ctypes.data, W, H, C.c_float(gamma), out.ctypes.data))
    return out


def rgb8_thresholds(gamma: float = 2.2):
    """The device quantiser's table: (thr (255,) float32, neg_mode); thr[k-1] = least
    float whose 8-bit value under to_rgb8 is >= k (pt_rgb8_thresholds)."""
    thr = np.empty(255, dtype=np.float32)
    mode = C.c_int32()
    check(lib().pt_rgb8_thresholds(C.c_float(gamma), thr.ctypes.data, C.byref(mode)))
    return thr, mode.value


def device_rgb8(img: np.ndarray, gamma: float = 2.2, device: int = 0) -> np.ndarray:
    """to_rgb8 computed by the device quantiser (test hook pt_debug_rgb8)."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    H, W = img.shape[:2]
    out = np.empty((H, W, 3), dtype=np.uint8)
    check(lib().pt_debug_rgb8(device, img.ctypes.data, W, H, C.c_float(gamma), out.ctypes.data))
    return out


def save_png(img: np.ndarray, filename: str, gamma: float = 2.2) -> bool:
    rgb = to_rgb8(img, gamma)
    rc = lib().pt_write_png(filename.encode(), rgb.ctypes.data, rgb.shape[1], rgb.shape[0])
    if rc < 0:
        print(lib().pt_last_error().decode(), file=sys.stderr)
        return False
    return True


def _render_to_file(camera: Camera, bvh: BVH, samples: int, depth: int, filename: str, unit: str, total: int,
                    after_done: str) -> bool:
    """render.h:62-104 / 109-152 around the device render: the reference's console lines
    (per row / per chunk progress as the library reports it, "Done in", "Saved to"), the
    image gamma-corrected and quantised on the device, its bytes written as the PNG."""
    if bvh.empty():
        print("No triangles in scene.", file=sys.stderr)
        return False
    if not bvh.built:
        print("Bounding volume heirarchy not built.\nBuilding...", file=sys.stderr)
        bvh.build()
    t0 = time.perf_counter()
    print(f"Rendered: 0/{total} {unit}.", end="", flush=True)
    printed = [0]

    def advance(k):
        while printed[0] < min(k, total):
            printed[0] += 1
            print(f"\rRendered: {printed[0]}/{total} {unit}.", end="", flush=True)

    rgb, _ = render_rgb8(camera, bvh, samples, depth, visible_devices(),
                         progress=lambda done, tot: advance(done * total // tot if tot else total))
    advance(total)
    print(f"\nDone in {math.floor((time.perf_counter() - t0) * 1000) / 1000:.2f} seconds.{after_done}")
    rc = lib().pt_write_png(filename.encode(), rgb.ctypes.data, rgb.shape[1], rgb.shape[0])
    if rc < 0:
        print(f"Failed to write image to file: {filename}", file=sys.stderr)
    print(f"Saved to {filename}")
    return True


def render_cpu(camera: Camera, bvh: BVH, samples: int, depth: int, filename: str) -> bool:
    """render.h:62-104 signature; the trace loop runs on the GPU."""
    return _render_to_file(camera, bvh, samples, depth, filename, "rows", camera.res[1], "\nColor correcting...")


def render_gpu(camera: Camera, bvh: BVH, samples: int, depth: int, chunk_size: Sequence[int], filename: str) -> bool:
    """render.h:109-152 signature; `chunk_size` only sets the progress granularity
    (the persistent kernel needs no watchdog-sized tiles)."""
    cx, cy = (chunk_size, chunk_size) if isinstance(chunk_size, int) else tuple(chunk_size)
    chunks = -(-camera.res[0] // cx) * -(-camera.res[1] // cy)
    return _render_to_file(camera, bvh, samples, depth, filename, "chunks", chunks, "")
