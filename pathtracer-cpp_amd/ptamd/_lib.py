"""ctypes binding of libpt_hip.so (C ABI declared in include/pt_hip.h).

The library is built in-tree (``make -C pathtracer-cpp_amd``); loading fails
loudly when it is missing — there is no fallback implementation.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import subprocess
from typing import Optional

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # pathtracer-cpp_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("PT_LIB") or os.path.join(PKG_ROOT, "lib", "libpt_hip.so")

PT_OK, PT_E_ARG, PT_E_EMPTY, PT_E_HIP, PT_E_IO, PT_E_RUNAWAY = 0, -1, -2, -3, -4, -5
PT_SEED = 1
PT_MAX_DEPTH = 64

EXPORTED = (
    "pt_abi_version", "pt_last_error", "pt_device_count", "pt_bvh_build", "pt_camera_init",
    "pt_ctx_create", "pt_ctx_destroy", "pt_ctx_set_scene", "pt_ctx_prepare", "pt_rtc_wait", "pt_ctx_render", "pt_part_rows",
    "pt_render_f32", "pt_image_to_rgb8", "pt_write_png", "pt_debug_math", "pt_debug_sweep", "pt_scene_validate", "pt_rtc_check",
    "pt_ctx_render_progressive", "pt_ctx_render_rgb8", "pt_rgb8_thresholds", "pt_debug_rgb8",
    "pt_obj_load", "pt_obj_num_tris", "pt_obj_triangles", "pt_obj_warnings", "pt_obj_free",
    "pt_render_f32_devices", "pt_render_rgb8_devices", "pt_scene_info", "pt_debug_wide_verify",
    "pt_debug_rccl_failover", "pt_debug_rtc_cache", "pt_devices_release", "pt_debug_ctx_flags", "pt_debug_counter",
    "pt_debug_scene_dark", "pt_debug_rtc_start", "pt_debug_pack_hash",
)
PT_MAX_DEVICES = 16


class pt_bvh_node(C.Structure):
    _fields_ = [("lb", C.c_float * 3), ("rt", C.c_float * 3), ("left", C.c_int32), ("right", C.c_int32),
                ("tri_start", C.c_int32), ("tri_end", C.c_int32)]


class pt_material(C.Structure):
    _fields_ = [("type", C.c_int32), ("color", C.c_float * 3), ("emit", C.c_float * 3), ("roughness", C.c_float)]


class pt_scene(C.Structure):
    _fields_ = [("num_tris", C.c_int32), ("verts", C.c_void_p), ("materials", C.c_void_p),
                ("num_nodes", C.c_int32), ("nodes", C.c_void_p), ("tri_idx", C.c_void_p)]


class pt_camera(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("res", C.c_int32 * 2), ("v_res", C.c_float * 2), ("cell_size", C.c_float),
                ("distance", C.c_float), ("transform", C.c_float * 9)]


class pt_params(C.Structure):
    _fields_ = [("spp", C.c_int32), ("depth", C.c_int32), ("seed", C.c_uint32), ("part_index", C.c_int32),
                ("part_count", C.c_int32), ("band_rows", C.c_int32), ("batch_spp", C.c_int32),
                ("samples_per_item", C.c_int32), ("progress", C.c_void_p), ("progress_user", C.c_void_p)]


class pt_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("paths", C.c_uint64), ("runaway", C.c_uint64), ("kernel_ms", C.c_double),
                ("reduce_ms", C.c_double), ("total_ms", C.c_double), ("trace_launches", C.c_int32),
                ("rows", C.c_int32), ("kernel_path", C.c_int32), ("n_devices", C.c_int32),
                ("gather_path", C.c_int32), ("gather_ms", C.c_double),
                ("device_kernel_ms", C.c_double * PT_MAX_DEVICES), ("device_render_ms", C.c_double * PT_MAX_DEVICES),
                ("device_rays", C.c_uint64 * PT_MAX_DEVICES)]

    PATHS = {0: "pt_trace_kernel<false,false> (tree, global)", 1: "pt_trace_kernel<true,false> (tree, LDS)",
             2: "pt_trace_kernel<true,true> (flat, table)", 3: "pt_trace_flat_rtc (flat, hipRTC-specialised)",
             4: "pt_trace_kernel<false,false,W> (wide tree, global)",
             5: "pt_flat_fast_kernel (flat, table with the scene's flags)"}

    GATHERS = {0: "none", 1: "rccl", 2: "host", 3: "host (RCCL unavailable or failed)"}

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_}
        n = max(self.n_devices, 0)
        for k in ("device_kernel_ms", "device_render_ms", "device_rays"):
            d[k] = list(d[k])[:n]
        return d


assert C.sizeof(pt_bvh_node) == 40 and C.sizeof(pt_material) == 32


class PTError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (code {code})")
        self.code = code


_lib: Optional[C.CDLL] = None


def build(force: bool = False) -> str:
    """Compile libpt_hip.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", PKG_ROOT], check=True)
    return LIB_PATH


def _torch_runtime_first() -> None:
    """PyTorch-ROCm wheels bundle their own HIP runtime (torch/lib/libamdhip64.so, no
    SONAME); libpt_hip.so links the system one (/opt/rocm). With both in one process,
    torch.cuda fails ("No HIP GPUs are available") when the system runtime initialised the
    devices first, while the other order works. So when torch is installed its runtime is
    brought up first (import + device count), and the two coexist."""
    import importlib.util
    if importlib.util.find_spec("torch") is None:
        return
    import torch
    torch.cuda.device_count()


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libpt_hip.so not built at {LIB_PATH}: run `make -C pathtracer-cpp_amd` "
                               "(there is no CPU fallback)")
        _torch_runtime_first()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.pt_abi_version.restype = C.c_int
        L.pt_last_error.restype = C.c_char_p
        L.pt_device_count.restype = C.c_int
        L.pt_bvh_build.argtypes = [C.c_int32, P, P, P]
        L.pt_camera_init.argtypes = [P, P, P, C.c_int32, C.c_int32, C.c_float, C.c_float, C.POINTER(pt_camera)]
        L.pt_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.pt_ctx_destroy.argtypes = [P]
        L.pt_ctx_destroy.restype = None
        L.pt_ctx_set_scene.argtypes = [P, C.POINTER(pt_scene)]
        L.pt_ctx_prepare.argtypes = [P]
        L.pt_rtc_wait.argtypes = []
        L.pt_rtc_wait.restype = C.c_int
        # no background compile left running into interpreter finalisation (pt_rtc_wait)
        atexit.register(L.pt_rtc_wait)
        L.pt_ctx_render.argtypes = [P, C.POINTER(pt_camera), C.POINTER(pt_params), P, C.c_int, C.POINTER(pt_stats)]
        L.pt_part_rows.argtypes = [C.c_int32] * 4
        L.pt_part_rows.restype = C.c_int32
        L.pt_render_f32.argtypes = [C.POINTER(pt_scene), C.POINTER(pt_camera), C.POINTER(pt_params), P,
                                    C.POINTER(pt_stats)]
        L.pt_image_to_rgb8.argtypes = [P, C.c_int32, C.c_int32, C.c_float, P]
        L.pt_write_png.argtypes = [C.c_char_p, P, C.c_int32, C.c_int32]
        L.pt_debug_math.argtypes = [C.c_int, C.c_int, P, C.c_int, P]
        L.pt_debug_sweep.argtypes = [C.c_int, C.c_int, C.c_uint32, C.c_uint32, P, P]
        L.pt_ctx_render_progressive.argtypes = [P, C.POINTER(pt_camera), C.POINTER(pt_params), C.c_int32,
                                                C.c_int32, P, C.c_int, C.POINTER(pt_stats)]
        L.pt_ctx_render_rgb8.argtypes = [P, C.POINTER(pt_camera), C.POINTER(pt_params), C.c_float, C.c_int, P,
                                         C.c_int, C.POINTER(pt_stats)]
        L.pt_rgb8_thresholds.argtypes = [C.c_float, P, P]
        L.pt_debug_rgb8.argtypes = [C.c_int, P, C.c_int32, C.c_int32, C.c_float, P]
        L.pt_render_f32_devices.argtypes = [C.POINTER(pt_scene), C.POINTER(pt_camera), C.POINTER(pt_params), P,
                                            C.c_int32, P, C.POINTER(pt_stats)]
        L.pt_render_rgb8_devices.argtypes = [C.POINTER(pt_scene), C.POINTER(pt_camera), C.POINTER(pt_params), P,
                                             C.c_int32, C.c_float, P, C.POINTER(pt_stats)]
        L.pt_obj_load.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]
        L.pt_obj_num_tris.argtypes = [P]
        L.pt_obj_num_tris.restype = C.c_int32
        L.pt_obj_triangles.argtypes = [P, P, P, P]
        L.pt_obj_warnings.argtypes = [P]
        L.pt_obj_warnings.restype = C.c_char_p
        L.pt_obj_free.argtypes = [P]
        L.pt_obj_free.restype = None
        L.pt_scene_validate.argtypes = [C.POINTER(pt_scene), P]
        L.pt_scene_info.argtypes = [C.POINTER(pt_scene), P, C.c_int32]
        L.pt_debug_wide_verify.argtypes = [C.POINTER(pt_scene), C.c_int32]
        L.pt_rtc_check.argtypes = [C.POINTER(pt_scene), C.c_char_p, C.c_size_t]
        if hasattr(L, "pt_debug_rccl_failover"):  # test hooks (absent from older builds used in A/B runs)
            L.pt_debug_rccl_failover.argtypes = [C.c_int32, C.c_int32, P]
        if hasattr(L, "pt_debug_rtc_cache"):
            L.pt_debug_rtc_cache.argtypes = [C.c_int32]
            L.pt_debug_rtc_cache.restype = C.c_int64
        if hasattr(L, "pt_devices_release"):
            L.pt_devices_release.argtypes = []
            L.pt_devices_release.restype = None
        if hasattr(L, "pt_debug_ctx_flags"):
            L.pt_debug_ctx_flags.argtypes = [P, P]
        if hasattr(L, "pt_debug_scene_dark"):
            L.pt_debug_scene_dark.argtypes = [C.POINTER(pt_scene)]
        if hasattr(L, "pt_debug_pack_hash"):
            L.pt_debug_pack_hash.argtypes = [C.POINTER(pt_scene), C.POINTER(C.c_uint64)]
        if hasattr(L, "pt_debug_rtc_start"):
            L.pt_debug_rtc_start.argtypes = [C.POINTER(pt_scene)]
        if hasattr(L, "pt_debug_counter"):
            L.pt_debug_counter.argtypes = [C.c_int32]
            L.pt_debug_counter.restype = C.c_int64
        if L.pt_abi_version() != 3:
            raise RuntimeError("libpt_hip.so ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int) -> int:
    if rc < 0:
        raise PTError(rc, lib().pt_last_error().decode(errors="replace"))
    return rc
