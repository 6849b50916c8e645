"""The C++ drop-in boundary: the reference's own programs compile unchanged
against pathtracer-cpp_amd/pathtracer/pathtracer.h, and renders through the
C++ API are bit-identical to the reference."""
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import ROOT, load_golden, scene_for

REF = "/root/reference"
PKG = os.path.join(ROOT, "pathtracer-cpp_amd")
TOOL = os.path.join(PKG, "bin", "pt_render_scene")
REF_OUT = os.path.join(ROOT, "oracle", "_ref")


@pytest.mark.skipif(not os.path.isdir(REF + "/examples"), reason="reference sources not present")
@pytest.mark.parametrize("src", ["examples/cornell_box.cc", "examples/modified_cornell.cc", "tests/test_render.cc"])
def test_reference_programs_compile_unchanged(src, tmp_path):
    import ptamd
    ptamd.build()
    out = tmp_path / "prog"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I" + PKG, "-I" + os.path.join(ROOT, "include"),
                        os.path.join(REF, src), "-L" + os.path.join(PKG, "lib"), "-lpt_hip", "-o", str(out)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def test_dropin_headers_compile_in_two_translation_units(tmp_path):
    """Unlike the reference's headers, the drop-in ones are ODR-safe (inline)."""
    a = tmp_path / "a.cc"
    b = tmp_path / "b.cc"
    a.write_text('#include "pathtracer/pathtracer.h"\nint f() { BVH b; return (int)b.size(); }\n')
    b.write_text('#include "pathtracer/pathtracer.h"\nint f();\nint main() { return f() + (int)rng.rand01(); }\n')
    r = subprocess.run(["g++", "-std=c++17", "-I" + PKG, "-I" + os.path.join(ROOT, "include"), str(a), str(b),
                        "-L" + os.path.join(PKG, "lib"), "-lpt_hip", "-o", str(tmp_path / "ab")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def _run_tool(scene, spp, depth):
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "s.ptscene")
        open(sp, "w").write(scene.to_ptscene())
        out = os.path.join(td, "o.f32")
        W, H = scene.camera.res
        r = subprocess.run([TOOL, sp, str(spp), str(depth), out], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        return np.fromfile(out, np.float32).reshape(H, W, 3), json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell_64_s16_d5", "mcornell_r0.3_64_s8_d5", "tri3_33x17_s5_d2"])
def test_cpp_api_render_bitexact(golden_meta, name):
    m = golden_meta["images"][name]
    img, meta = _run_tool(scene_for(m["scene"], m["res"]), m["spp"], m["depth"])
    ref = load_golden(name)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    assert meta["rays"] > 0


@pytest.mark.gpu
@pytest.mark.skipif(not os.access(os.path.join(REF_OUT, "dropin_test_render"), os.X_OK),
                    reason="oracle/_ref/dropin_test_render not built")
def test_reference_test_render_program_runs_on_gpu(tmp_path):
    """tests/test_render.cc of the reference, compiled against the drop-in: both of its
    renders (render_gpu and render_cpu, 512^2, 500 spp, depth 5) go through the GPU
    kernel; the PNGs it writes decode to the Python path's gamma-corrected pixels."""
    from PIL import Image as PILImage
    import ptamd
    from ptamd import scenes
    prefix = str(tmp_path / "tr")
    r = subprocess.run([os.path.join(REF_OUT, "dropin_test_render"), prefix], capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    stdout = r.stdout.decode()  # bytes: text mode would turn the progress lines' \r into \n
    # the reference's console contract (render.h:127-149, then 79-101) byte for byte, but
    # for the timings: every per-chunk and per-row progress line, in order
    import re
    want = ("Rendered: 0/9 chunks." + "".join(f"\rRendered: {k}/9 chunks." for k in range(1, 10)) +
            "\nDone in T seconds.\nSaved to " + prefix + ".gpu.png\n" +
            "Rendered: 0/512 rows." + "".join(f"\rRendered: {k}/512 rows." for k in range(1, 513)) +
            "\nDone in T seconds.\nColor correcting...\nSaved to " + prefix + ".cpu.png\n")
    got = re.sub(r"Done in \d+\.\d\d seconds", "Done in T seconds", stdout)
    if got != want:
        i = next((k for k in range(min(len(got), len(want))) if got[k] != want[k]), min(len(got), len(want)))
        raise AssertionError(f"stdout differs at {i}: got {got[max(0, i - 40):i + 80]!r} want {want[max(0, i - 40):i + 80]!r}")
    sc = scenes.tri3((512, 512))
    img, _ = ptamd.render(ptamd.Camera.from_spec(sc.camera), ptamd.BVH.from_scene(sc), 500, 5)
    want = ptamd.to_rgb8(img)
    for suffix in (".gpu.png", ".cpu.png"):
        got = np.asarray(PILImage.open(prefix + suffix).convert("RGB"))
        assert np.array_equal(got, want), suffix


def test_dropin_load_obj_matches_reference(tmp_path):
    """BVH::load_obj of the drop-in header (through pt_obj_load) loads the same
    triangles and Material bytes as the reference's tinyobjloader path."""
    obj_dir = os.path.join(ROOT, "tests", "golden", "obj")
    src = tmp_path / "lo.cc"
    src.write_text(
        '#include "pathtracer/pathtracer.h"\n#include <cstdio>\n'
        'int main(int argc, char** argv) {\n'
        '    BVH b; b.load_obj(argv[1], argv[2]);\n'
        '    FILE* f = std::fopen(argv[3], "wb");\n'
        '    for (const Triangle& t : b.triangles) {\n'
        '        const float v[9] = {t.v1.x, t.v1.y, t.v1.z, t.v2.x, t.v2.y, t.v2.z, t.v3.x, t.v3.y, t.v3.z};\n'
        '        std::fwrite(v, 4, 9, f); std::fwrite(&t.material, 32, 1, f);\n'
        '    }\n'
        '    std::fclose(f);\n'
        '    try { BVH c; c.load_obj(std::string(argv[2]) + "/nomtl.obj", argv[2]); } '
        'catch (const std::runtime_error& e) { std::printf("threw: %s\\n", e.what()); }\n'
        '}\n')
    exe = tmp_path / "lo"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-I" + PKG, "-I" + os.path.join(ROOT, "include"), str(src),
                        "-L" + os.path.join(PKG, "lib"), "-lpt_hip", "-Wl,-rpath," + os.path.join(PKG, "lib"),
                        "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    for name in ("edge", "polys"):
        out = tmp_path / (name + ".bin")
        r = subprocess.run([str(exe), os.path.join(obj_dir, name + ".obj"), obj_dir, str(out)],
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "threw: load_obj: a face has no material" in r.stdout
        rec = np.fromfile(str(out), np.uint8).reshape(-1, 68)
        assert rec[:, :36].tobytes() == load_golden(f"obj_{name}_verts").tobytes()
        assert rec[:, 36:].tobytes() == load_golden(f"obj_{name}_mats").tobytes()
        assert r.stderr.count("Unknown material type with illum") == (4 if name == "edge" else 0)


@pytest.mark.gpu
def test_cpp_api_render_over_listed_devices(golden_meta, monkeypatch):
    """The drop-in renders over every device PT_DEVICES lists (here the box's one GPU
    twice: two contexts, two host threads) with the same bits."""
    monkeypatch.setenv("PT_DEVICES", "0,0")
    m = golden_meta["images"]["cornell_64_s16_d5"]
    img, _ = _run_tool(scene_for(m["scene"], m["res"]), m["spp"], m["depth"])
    assert np.array_equal(img.view(np.uint32), load_golden("cornell_64_s16_d5").view(np.uint32))
