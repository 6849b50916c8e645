#!/usr/bin/env python3
"""Scene-kernel compile times on this host (round 6, cold-start analysis; no GPU work).

Each mode runs in a fresh process that first initialises the GPU through torch (as bench.py
does), then compiles Cornell's and modified Cornell's scene kernels with pt_rtc_check on an
empty code-object cache: through the compile server (default) or in this process
(PT_RTC_SERVER=0), and, for reference, a trivial kernel straight through the process's hipRTC
twice (its one-time initialisation). Prints one JSON line per mode.
usage: python scripts/rtc_timing.py [--child MODE]
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(mode):
    import ctypes as C
    import torch
    if torch.cuda.is_available():
        torch.zeros(1, device="cuda").sum().item()
    sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))
    import ptamd
    from ptamd import scenes
    L = ptamd.lib()
    out = {"mode": mode}
    if mode == "direct_trivial":
        # the hipRTC this process's library resolved (PyTorch's when torch is loaded)
        maps = open("/proc/self/maps").read().split("\n")
        path = next(l.split()[-1] for l in maps if "libhiprtc" in l)
        out["hiprtc"] = path
        R = C.CDLL(path)
        prog = C.c_void_p()
        opts = [b"--offload-arch=gfx950", b"-O3"]
        for k in range(2):
            assert R.hiprtcCreateProgram(C.byref(prog), b'extern "C" __global__ void k(float* p) { p[threadIdx.x] = 1.0f; }',
                                         b"t.hip", 0, None, None) == 0
            t = time.perf_counter()
            rc = R.hiprtcCompileProgram(prog, len(opts), (C.c_char_p * len(opts))(*opts))
            out[f"trivial_{k}_s"] = time.perf_counter() - t
            assert rc == 0
        print(json.dumps(out), flush=True)
        return
    for name, sc in (("cornell", scenes.cornell((16, 16))), ("mcornell", scenes.modified_cornell(0.3, (16, 16)))):
        ref = ptamd._SceneRef(ptamd.BVH.from_scene(sc))
        t = time.perf_counter()
        n = L.pt_rtc_check(C.byref(ref.s), None, 0)
        out[name + "_s"] = time.perf_counter() - t
        out[name + "_compile_s"] = L.pt_debug_rtc_cache(4) / 1e6
        assert n > 0, L.pt_last_error()
    out["server_compiles"] = L.pt_debug_rtc_cache(5)
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    for mode, env in (("server", {}), ("in_process", {"PT_TEST_HOOKS": "1", "PT_RTC_SERVER": "0"}),
                      ("server", {}), ("in_process", {"PT_TEST_HOOKS": "1", "PT_RTC_SERVER": "0"}),
                      ("direct_trivial", {})):
        with tempfile.TemporaryDirectory() as d:
            e = dict(os.environ, PT_RTC_CACHE_DIR=d, **env)
            r = subprocess.run([sys.executable, __file__, "--child", mode], env=e, capture_output=True, text=True,
                               timeout=300)
            print(r.stdout.strip() if r.returncode == 0 else json.dumps({"mode": mode, "rc": r.returncode,
                                                                       "err": r.stderr[-400:]}), flush=True)


if __name__ == "__main__":
    main()
