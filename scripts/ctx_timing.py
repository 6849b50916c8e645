#!/usr/bin/env python3
"""Cold-start accounting on the GPU box: wall time of each step between an initialised torch
device and the first finished frame (library load, context phases via PT_TIME_CTX, scene
upload, first and second small renders, a second context). One JSON line on stdout."""
import json
import os
import sys
import time

os.environ.setdefault("PT_TEST_HOOKS", "1")
os.environ.setdefault("PT_TIME_CTX", "1")
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))
torch.zeros(1, device="cuda").sum().item()
out = {}


def tick(name, fn):
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    out[name] = round((time.perf_counter() - t0) * 1e3, 3)
    return r


ptamd = tick("import_ptamd_ms", lambda: __import__("ptamd"))
from ptamd import scenes  # noqa: E402

tick("lib_load_ms", ptamd.lib)
bvh = tick("bvh_build_ms", lambda: ptamd.BVH.from_scene(scenes.cornell((1024, 1024))))
cam = ptamd.Camera.from_spec(scenes.cornell((1024, 1024)).camera)
r = tick("ctx_create_ms", lambda: ptamd.Renderer(0))
tick("set_scene_ms", lambda: r.set_scene(bvh))
tick("first_render_1spp_ms", lambda: r.render(cam, 1, 5))
tick("second_render_1spp_ms", lambda: r.render(cam, 1, 5))
tick("prepare_ms", r.prepare)
tick("third_render_1spp_ms", lambda: r.render(cam, 1, 5))
r2 = tick("second_ctx_create_ms", lambda: ptamd.Renderer(0))
r2.close()
r.close()
print(json.dumps(out))
