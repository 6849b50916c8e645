"""Where pt_ctx_create's time goes (first vs second context in a process; torch already
initialised, as in bench.py). Prints one line per phase."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pathtracer-cpp_amd"))
import torch
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
torch.cuda.synchronize()
import ptamd
from ptamd import scenes
t = time.perf_counter(); ptamd.lib(); print("lib load %.1f ms" % ((time.perf_counter() - t) * 1e3))
for i in range(3):
    t = time.perf_counter(); r = ptamd.Renderer(0); print("context %d: %.1f ms" % (i, (time.perf_counter() - t) * 1e3))
    sc = scenes.cornell((64, 64)); bvh = ptamd.BVH.from_scene(sc); bvh.build()
    t = time.perf_counter(); r.set_scene(bvh); torch.cuda.synchronize(); print("  set_scene %.1f ms" % ((time.perf_counter() - t) * 1e3))
    cam = ptamd.Camera.from_spec(sc.camera)
    t = time.perf_counter(); r.render(cam, 4, 5); print("  first render %.1f ms" % ((time.perf_counter() - t) * 1e3))
    t = time.perf_counter(); r.render(cam, 4, 5); print("  second render %.1f ms" % ((time.perf_counter() - t) * 1e3))
    r.close()
