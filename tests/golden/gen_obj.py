"""OBJ/MTL ingestion fixtures (BVH::load_obj, bvh.h:184-242).

Writes the input files under tests/golden/obj/ (hand-written edge cases plus seeded
random number formats, polygons and a renderable mesh), then runs the reference
harness (oracle/_ref/pt_ref, built from /root/reference by oracle/ref/build_ref.sh;
load_obj -> the reference's vendored tinyobjloader) on each and stores what it loaded:
  obj_<name>_verts.npy  (n, 9) float32   v1, v2, v3 of every triangle, in load order
  obj_<name>_mats.npy   (n, 32) uint8    the reference's Material bytes
  obj_<name>_nodes.npy / _idx.npy        the reference's BVH::build of those triangles
  obj_mesh_img.npy                       a render of mesh.obj (res/spp/depth in golden.json)
Run from the repo root: python tests/golden/gen_obj.py
"""
from __future__ import annotations

import json
import math
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OBJ_DIR = os.path.join(HERE, "obj")
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _oracle as O  # noqa: E402

# Camera of examples/cornell_box.cc (used to render mesh.obj).
CAMERA = "camera 278.0 278.0 -500.0 0.0 0.0 1.0 0.0 1.0 0.0 {w} {h} 60.0 1.0\n"
MESH_RENDER = dict(res=[48, 48], spp=8, depth=5)

EDGE_OBJ = """\
# hand-written edge cases of the reader
mtllib missing.mtl edge.mtl
mtllib lib2.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v +2.5 -.5 1e1
v 3.25E-1 .75 -0
v 1.000000001 2.00000000000000000001 123456789012
v 7. -8.e2 0.1234567890123
v 1e-40 -1e30 5
v 1.5e 2x 3
v 4 5
v\t0.5\t0.25\t-0.125
v 1 -2 0
vt 0 0
vn 0 0 1
usemtl white
f 1 2 3
f 1/1 3/1 4/1
f 1//1 2//1 3//1
f 1/1/1 2/1/1 4/1/1
l 1 2
p 3
usemtl light
f -4 -3 -2
f 1 2 3 4
f 1 14 2 4
g group one
usemtl other
f 2 3 4 5 6
o second
usemtl white
f 9 10 11
usemtl dflt
f 1 3 5
usemtl spec\r
f 2 4 6\r
usemtl kdmap
   f 3 5 7   \t
usemtl white
usemtl white
f 12 13 1
f 1 2 3 4 5 6 7 8
"""

EDGE_MTL = """\
# materials; Kd here sets LoadMtl's has_kd for the whole file
newmtl white
Kd 0.75 0.5 .25
illum 1
newmtl light
Ka 4 3.5 +2e0
Kd 1 1 1
illum 2
newmtl other
Kd 0.1 0.2 0.3
illum 3
newmtl dflt
Kd 0.9 0.9 0.9
newmtl spec
Ka 1 1 1
  illum 2   \t
"""

LIB2_MTL = """\
newmtl kdmap
map_Kd texture.png
illum 1
newmtl white
Kd 0 0 1
illum 1
"""


def _fmt(rng, x: float) -> str:
    """x in one of the textual forms OBJ exporters write (and a few they should not)."""
    k = int(rng.integers(0, 12))
    if k == 0:
        return repr(x)
    if k == 1:
        return "%.*f" % (int(rng.integers(0, 21)), x)
    if k == 2:
        return "%.*e" % (int(rng.integers(0, 18)), x)
    if k == 3:
        return ("%.*E" % (int(rng.integers(0, 18)), x)).replace("E", "E+" if rng.random() < 0.3 else "E")
    if k == 4:
        s = "%.9f" % x
        return s.replace("0.", ".", 1) if s.startswith(("0.", "-0.")) else s
    if k == 5:
        return ("+" if x >= 0 else "") + "%.6f" % x
    if k == 6:
        return "%d." % int(x)
    if k == 7:
        return "%d" % int(x * 1e6) + "e-6"
    if k == 8:
        return "%.30f" % x
    if k == 9:
        return "%.17g" % x
    if k == 10:
        return "%.3g" % x
    return "%.12f" % x


def numbers_obj(rng) -> str:
    lines = ["mtllib numbers.mtl", "usemtl m"]
    n = 3000
    for _ in range(n):
        vals = [math.copysign(10 ** rng.uniform(-8, 8), rng.random() - 0.5) for _ in range(3)]
        lines.append("v " + " ".join(_fmt(rng, float(x)) for x in vals))
    for i in range(0, n, 3):
        lines.append(f"f {i + 1} {i + 2} {i + 3}")
    return "\n".join(lines) + "\n"


def polys_obj(rng) -> str:
    """Random planar and non-planar polygons of 5-12 corners in random orientations
    (convex, star-shaped and shuffled corner orders) for the ear-clipping restatement."""
    lines = ["mtllib numbers.mtl", "usemtl m"]
    nv = 0
    for p in range(400):
        n = int(rng.integers(5, 13))
        ang = np.sort(rng.uniform(0, 2 * np.pi, n))
        rad = rng.uniform(0.2, 1.0, n) if p % 3 else np.ones(n)
        pts2 = np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1)
        if p % 7 == 0:
            pts2 = pts2[rng.permutation(n)]
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        if p % 5 == 0:
            q = np.eye(3)[rng.permutation(3)]  # axis-aligned planes
        pts = pts2 @ q[:2] + rng.normal(size=3) * 5
        if p % 4 == 0:
            pts = pts + rng.normal(size=(n, 3)) * 0.05  # non-planar
        for x in pts.astype(np.float32):
            lines.append("v " + " ".join(repr(float(c)) for c in x))
        lines.append("f " + " ".join(str(nv + 1 + k) for k in range(n)))
        nv += n
    return "\n".join(lines) + "\n"


NUMBERS_MTL = "newmtl m\nKd 0.5 0.5 0.5\nillum 1\n"


def mesh_obj() -> tuple:
    """Cornell room as quads + a UV sphere with polygon pole caps (ear clipping)."""
    lines = ["mtllib mesh.mtl"]
    vs = []

    def v(p):
        vs.append(p)
        lines.append("v " + " ".join(repr(float(c)) for c in p))
        return len(vs)

    def quad(a, b, c, d, mat):
        ids = [v(a), v(b), v(c), v(d)]
        lines.append(f"usemtl {mat}")
        lines.append("f " + " ".join(map(str, ids)))

    S = 555.0
    quad((0, 0, 0), (S, 0, 0), (S, 0, S), (0, 0, S), "white")        # floor
    quad((0, S, 0), (0, S, S), (S, S, S), (S, S, 0), "white")        # ceiling
    quad((0, 0, S), (S, 0, S), (S, S, S), (0, S, S), "white")        # back
    quad((0, 0, 0), (0, 0, S), (0, S, S), (0, S, 0), "red")          # left
    quad((S, 0, 0), (S, S, 0), (S, S, S), (S, 0, S), "green")        # right
    quad((213, S - 1, 227), (343, S - 1, 227), (343, S - 1, 332), (213, S - 1, 332), "light")
    st, sl, r, c = 8, 10, 110.0, (278.0, 160.0, 300.0)
    lines.append("usemtl grey")
    rings = []
    for i in range(1, st):
        th = math.pi * i / st
        rings.append([v((c[0] + r * math.sin(th) * math.cos(2 * math.pi * j / sl),
                         c[1] + r * math.cos(th),
                         c[2] + r * math.sin(th) * math.sin(2 * math.pi * j / sl))) for j in range(sl)])
    lines.append("f " + " ".join(str(k) for k in rings[0]))             # top cap polygon
    for a, b in zip(rings[:-1], rings[1:]):
        for j in range(sl):
            lines.append(f"f {a[j]} {b[j]} {b[(j + 1) % sl]} {a[(j + 1) % sl]}")
    lines.append("f " + " ".join(str(k) for k in reversed(rings[-1])))  # bottom cap polygon
    mtl = ("newmtl white\nKd 0.73 0.73 0.73\nillum 1\nnewmtl red\nKd 0.65 0.05 0.05\nillum 1\n"
           "newmtl green\nKd 0.12 0.45 0.15\nillum 1\nnewmtl light\nKa 15 15 15\nillum 2\n"
           "newmtl grey\nKd 0.8 0.8 0.8\nillum 1\n")
    return "\n".join(lines) + "\n", mtl


def write_inputs() -> dict:
    os.makedirs(OBJ_DIR, exist_ok=True)
    rng = np.random.default_rng(20261016)
    mesh, mesh_mtl = mesh_obj()
    files = {"edge.obj": EDGE_OBJ, "edge.mtl": EDGE_MTL, "lib2.mtl": LIB2_MTL,
             "numbers.obj": numbers_obj(rng), "numbers.mtl": NUMBERS_MTL, "polys.obj": polys_obj(rng),
             "mesh.obj": mesh, "mesh.mtl": mesh_mtl,
             "nomtl.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n",
             "badidx.obj": "mtllib numbers.mtl\nusemtl m\nv 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 4\n",
             "zeroidx.obj": "mtllib numbers.mtl\nusemtl m\nv 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n"}
    for name, text in files.items():
        with open(os.path.join(OBJ_DIR, name), "w", newline="") as f:
            f.write(text)
    return files


def ref_load(obj: str, extra=(), res=(2, 2), spp=1, depth=1):
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "cam.ptscene")
        with open(sp, "w") as f:
            f.write(CAMERA.format(w=res[0], h=res[1]))
        tf, bf, of = (os.path.join(td, n) for n in ("tris.bin", "bvh.bin", "img.f32"))
        cmd = [O.REF_BIN, "--scene", sp, "--obj", os.path.join(OBJ_DIR, obj), "--mtl", OBJ_DIR,
               "--spp", str(spp), "--depth", str(depth), "--dump-tris", tf, "--dump-bvh", bf, "--out", of, *extra]
        r = subprocess.run(cmd, check=True, capture_output=True, text=True)
        raw = open(tf, "rb").read()
        n = int(np.frombuffer(raw[:4], np.int32)[0])
        rec = np.frombuffer(raw[4:], np.uint8).reshape(n, 68)
        verts = rec[:, :36].copy().view(np.float32).reshape(n, 9)
        mats = rec[:, 36:].copy()
        braw = open(bf, "rb").read()
        nn = int(np.frombuffer(braw[:4], np.int32)[0])
        nodes = np.frombuffer(braw[8:8 + 40 * nn], dtype=O.NODE_DTYPE)
        idx = np.frombuffer(braw[8 + 40 * nn:], np.int32)
        img = np.fromfile(of, np.float32).reshape(res[1], res[0], 3)
        return verts, mats, nodes, idx, img, r.stderr


def main() -> None:
    if not O.ref_available():
        subprocess.run([os.path.join(ROOT, "oracle", "ref", "build_ref.sh")], check=True)
    write_inputs()
    meta = {}
    for name in ("edge", "numbers", "polys", "mesh"):
        kw = dict(res=MESH_RENDER["res"], spp=MESH_RENDER["spp"], depth=MESH_RENDER["depth"]) if name == "mesh" else {}
        verts, mats, nodes, idx, img, err = ref_load(name + ".obj", **kw)
        np.save(os.path.join(HERE, f"obj_{name}_verts.npy"), verts)
        np.save(os.path.join(HERE, f"obj_{name}_mats.npy"), mats)
        np.save(os.path.join(HERE, f"obj_{name}_nodes.npy"), nodes)
        np.save(os.path.join(HERE, f"obj_{name}_idx.npy"), idx)
        meta[name] = dict(tris=int(verts.shape[0]), nodes=int(nodes.shape[0]),
                          unknown_material_msgs=err.count("Unknown material type with illum"))
        if name == "mesh":
            np.save(os.path.join(HERE, "obj_mesh_img.npy"), img)
            meta[name]["render"] = MESH_RENDER
        print(name, meta[name])
    gm = os.path.join(HERE, "golden.json")
    g = json.load(open(gm))
    g["obj"] = dict(generator="tests/golden/gen_obj.py", camera=CAMERA.strip(), files=meta)
    with open(gm, "w") as f:
        json.dump(g, f, indent=1)


if __name__ == "__main__":
    main()
