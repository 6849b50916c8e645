"""A process that exits while the scene kernel's hipRTC compile is still running (no GPU
needed: hipRTC compiles for gfx950 on any host).

Round 5 saw such exits die with SIGSEGV. The cause, reproduced here without a device
(DESIGN.md §3.9): a compile on a background thread of the render process runs inside
amd_comgr, whose lazily constructed statics register their destructors with atexit during
the compile — after the library's handler that waits for it — so exit() destroyed them
under the running compile (the faulting thread: a call through a destroyed object from
amd_comgr_do_action). The library now compiles in a child process (bin/pt_rtc_server); the
render process's exit only closes a socket. Both hosts below exit with a compile in flight
and without the Python package's own interpreter-exit wait."""
import os
import subprocess
import sys
import textwrap

import pytest

from conftest import ROOT

PKG = os.path.join(ROOT, "pathtracer-cpp_amd")

PY_PROG = textwrap.dedent("""
    import atexit, ctypes as C, sys
    sys.path.insert(0, %r)
    import ptamd
    from ptamd import scenes
    L = ptamd.lib()
    atexit.unregister(L.pt_rtc_wait)  # no interpreter-exit wait: the library alone must cope
    ref = ptamd._SceneRef(ptamd.BVH.from_scene(scenes.cornell((16, 16))))
    print("started", L.pt_debug_rtc_start(C.byref(ref.s)), flush=True)
""") % PKG

CPP_PROG = r"""
#include <cstdio>
#include "pathtracer/pathtracer.h"
#include "pt_hip_debug.h"
int main() {
    BVH bvh;
    const Material white(Material::DIFFUSE, vec3(1, 1, 1), vec3(0, 0, 0), 0.0f);
    const Material light(Material::EMIT, vec3(0, 0, 0), vec3(1, 1, 1), 0.0f);
    bvh.add_triangle(Triangle(vec3(0, 0, 0), vec3(1, 0, 0), vec3(0, 1, 0), white));
    bvh.add_triangle(Triangle(vec3(0, 0, 1), vec3(1, 0, 1), vec3(0, 1, 1), white));
    bvh.add_triangle(Triangle(vec3(0, 2, 0), vec3(1, 2, 0), vec3(0, 2, 1), light));
    bvh.build();
    const Camera cam(vec3(0.3f, 0.3f, -3), vec3(0, 0, 1), vec3(0, 1, 0), ivec2(8, 8), 60, 1);
    PtRenderCall call(cam, bvh, 1, 3, SEED);
    std::printf("started %d\n", pt_debug_rtc_start(&call.sc));
    return 0;  // exit with the compile in flight
}
"""


def _env(tmp_path, **extra):
    env = dict(os.environ)
    env["PT_RTC_CACHE_DIR"] = str(tmp_path / "cache")  # empty: the compile really runs
    env.update(extra)
    return env


@pytest.fixture(scope="module")
def built():
    import ptamd
    ptamd.build()
    assert os.access(os.path.join(PKG, "bin", "pt_rtc_server"), os.X_OK)


def _cache_entries(tmp_path):
    d = tmp_path / "cache"
    return sorted(p.name for p in d.iterdir()) if d.is_dir() else []


def test_python_exit_with_compile_in_flight(built, tmp_path):
    r = subprocess.run([sys.executable, "-X", "faulthandler", "-c", PY_PROG], env=_env(tmp_path),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == "started 1"  # the compile was still running at exit
    # the library's exit handler waited for the server's answer: the entry is in the cache
    assert len([n for n in _cache_entries(tmp_path) if n.endswith(".co")]) == 1


def test_cpp_program_exit_with_compile_in_flight(built, tmp_path):
    src = tmp_path / "exit_race.cc"
    src.write_text(CPP_PROG)
    exe = tmp_path / "exit_race"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-I" + PKG, "-I" + os.path.join(ROOT, "include"), str(src),
                        "-L" + os.path.join(PKG, "lib"), "-lpt_hip", "-Wl,-rpath," + os.path.join(PKG, "lib"),
                        "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([str(exe)], env=_env(tmp_path), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == "started 1"
    assert len([n for n in _cache_entries(tmp_path) if n.endswith(".co")]) == 1


def test_in_process_fallback_still_compiles(built, tmp_path):
    """PT_RTC_SERVER=0 (test hook): the compile runs in this process (the round-5 form, kept
    for hosts without the server binary) and gives the same code object size as the server."""
    prog = textwrap.dedent("""
        import ctypes as C, sys
        sys.path.insert(0, %r)
        import ptamd
        from ptamd import scenes
        ref = ptamd._SceneRef(ptamd.BVH.from_scene(scenes.cornell((16, 16))))
        print(ptamd.lib().pt_rtc_check(C.byref(ref.s), None, 0))
    """) % PKG
    sizes = []
    for server in ("1", "0"):
        r = subprocess.run([sys.executable, "-c", prog], env=_env(tmp_path / server, PT_TEST_HOOKS="1",
                                                                    PT_RTC_SERVER=server),
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        sizes.append(int(r.stdout.strip()))
    assert sizes[0] == sizes[1] > 0
