#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the UNMODIFIED reference.

Runs in the development container only (needs /root/reference to build
oracle/_ref/pt_ref; see oracle/ref/build_ref.sh). The committed outputs are data
(inputs + expected outputs); no reference source is stored.

Every fixture is produced by oracle/_ref/pt_ref — the reference's render.h:36-61
trace(), camera.h get_ray, bvh.h build/intersect and image.h accumulation,
compiled with g++ -O3 from /root/reference — driven with the per-sample reseed
of include/pt_hip.h (pt_sample_seed). Scenes come from ptamd/scenes.py; the
sha256 of each scene's .ptscene text is recorded so a scene edit invalidates the
fixture instead of silently changing it.

Usage: python tests/golden/gen_golden.py [--mesh | --png | --r3]
  --mesh  also (re)generate the config-4 fixtures for the 99,044-triangle sphere-in-Cornell
          mesh: sampled pixels at 1024^2 / 1k spp and the sha256 of the reference's BVH
          (the reference's O(n^2) BVH::build takes ~5.5 min here).
  --r3    only add the round-3 full-size pixel sets (config 3, r = 0 / 0.1 / 0.5 / 0.8).
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from ptamd import scenes  # noqa: E402
import _oracle as O  # noqa: E402

# (fixture name, scene factory, res, spp, depth)
IMAGES = [
    ("cornell_64_s16_d5", lambda r: scenes.cornell(r), (64, 64), 16, 5),
    ("cornell_64_s16_d3", lambda r: scenes.cornell(r), (64, 64), 16, 3),
    ("cornell_48x40_s8_d8", lambda r: scenes.cornell(r), (48, 40), 8, 8),
    ("cornell_256_s16_d3", lambda r: scenes.cornell(r), (256, 256), 16, 3),  # config 1, full
    ("mcornell_r0_64_s8_d5", lambda r: scenes.modified_cornell(0.0, r), (64, 64), 8, 5),
    ("mcornell_r0.3_64_s8_d5", lambda r: scenes.modified_cornell(0.3, r), (64, 64), 8, 5),
    ("mcornell_r0.8_64_s8_d5", lambda r: scenes.modified_cornell(0.8, r), (64, 64), 8, 5),
    ("tri3_64_s16_d5", lambda r: scenes.tri3(r), (64, 64), 16, 5),
    ("tri3_33x17_s5_d2", lambda r: scenes.tri3(r), (33, 17), 5, 2),
    ("cornell_16_s4_d1", lambda r: scenes.cornell(r), (16, 16), 4, 1),
]

# Full-size configs pinned at sampled pixels, full spp.
PIXEL_SETS = [
    ("cfg2_cornell_1024_s10000_d5_px", lambda: scenes.cornell((1024, 1024)), 10000, 5, 64),
    ("cfg3_mcornell_r0.3_1024_s10000_d5_px", lambda: scenes.modified_cornell(0.3, (1024, 1024)), 10000, 5, 12),
    ("cfg3_mcornell_r0.05_1024_s10000_d5_px", lambda: scenes.modified_cornell(0.05, (1024, 1024)), 10000, 5, 8),
    ("cfg5_cornell_4096_s10000_d8_px", lambda: scenes.cornell((4096, 4096)), 10000, 8, 8),
]

# Round 3: the other four roughness values of config 3 (modified_cornell.cc:14) at full size,
# 8 sampled pixels each (own pixel stream, so the sets above keep their pixels).
PIXEL_SETS_R3 = [
    (f"cfg3_mcornell_r{r}_1024_s10000_d5_px", (lambda r=r: scenes.modified_cornell(r, (1024, 1024))), 10000, 5, 8)
    for r in (0.0, 0.1, 0.5, 0.8)
]

BVHS = [
    ("bvh_cornell", lambda: scenes.cornell((64, 64))),
    ("bvh_mcornell", lambda: scenes.modified_cornell(0.3, (64, 64))),
    ("bvh_tri3", lambda: scenes.tri3((64, 64))),
]


def scene_hash(sc) -> str:
    """Hash of the geometry/materials/camera placement, resolution excluded."""
    return hashlib.sha256(sc.with_res(1, 1).to_ptscene().encode()).hexdigest()


def mesh_fixtures(meta) -> None:
    sc = scenes.sphere_in_cornell(223, (1024, 1024))
    rng = np.random.default_rng(4)
    px = [(int(rng.integers(0, 1024)), int(rng.integers(0, 1024))) for _ in range(16)]
    px += [(512, 560), (500, 430), (530, 470), (560, 520)]  # on the sphere
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "s.ptscene")
        with open(sp, "w") as f:
            f.write(sc.to_ptscene())
        pf = os.path.join(td, "px.txt")
        with open(pf, "w") as f:
            f.write("\n".join(f"{w} {h}" for w, h in px) + "\n")
        out, bvh = os.path.join(td, "px.f32"), os.path.join(td, "bvh.bin")
        r = subprocess.run([O.REF_BIN, "--scene", sp, "--spp", "1000", "--depth", "5", "--pixels", pf, "--out", out,
                            "--dump-bvh", bvh], check=True, capture_output=True, text=True)
        m = json.loads(r.stdout.strip().splitlines()[-1])
        vals = np.fromfile(out, dtype=np.float32).reshape(-1, 3)
        raw = open(bvh, "rb").read()
    name = "cfg4_sphere223_1024_s1000_d5_px"
    np.save(os.path.join(HERE, name + ".npy"), vals)
    meta["pixels"][name] = dict(scene=sc.name, scene_sha256=scene_hash(sc), res=[1024, 1024], spp=1000, depth=5,
                                pixels=px, ref_render_s=m["render_s"])
    nn = int(np.frombuffer(raw[:4], np.int32)[0])
    meta["bvh_hash"] = {"sphere223_in_cornell": dict(
        scene_sha256=scene_hash(sc), nodes=nn, ref_build_s=m["build_s"],
        sha256_nodes_then_tri_idx=hashlib.sha256(raw[8:]).hexdigest())}
    print(name, vals.shape, "ref BVH::build %.1f s" % m["build_s"])


PNGS = ["cornell_64_s16_d5", "cornell_48x40_s8_d8", "mcornell_r0.3_64_s8_d5"]


def png_fixtures(meta) -> None:
    """The reference's own PNG bytes (render.h:99-100 via pt_ref --png), decoded."""
    from PIL import Image as PILImage
    meta["png"] = {}
    for name in PNGS:
        m = meta["images"][name]
        sc = next(fac(tuple(m["res"])) for n, fac, *_ in IMAGES if n == name)
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "ref.png")
            img, _ = O.ref_run(sc, m["spp"], m["depth"], extra=["--png", p])
            assert img.tobytes() == np.load(os.path.join(HERE, name + ".npy")).tobytes(), name
            rgb = np.asarray(PILImage.open(p).convert("RGB"))
        np.save(os.path.join(HERE, name + "_png.npy"), rgb)
        meta["png"][name] = dict(image=name, gamma=2.2, shape=list(rgb.shape))
        print(name, "png", rgb.shape)


def pixel_sets(meta, sets, rng) -> None:
    for name, fac, spp, depth, n in sets:
        sc = fac()
        W, H = sc.camera.res
        px = [(int(rng.integers(0, W)), int(rng.integers(0, H))) for _ in range(n)]
        vals, m = O.ref_run(sc, spp, depth, pixels=px, timeout=3600)
        np.save(os.path.join(HERE, name + ".npy"), vals)
        meta["pixels"][name] = dict(scene=sc.name, scene_sha256=scene_hash(sc), res=[W, H], spp=spp, depth=depth,
                                    pixels=px, ref_render_s=m["render_s"])
        print(name, vals.shape, m["render_s"])


def main() -> None:
    if "--r3" in sys.argv:  # add the round-3 pixel sets to an existing golden.json
        meta = json.load(open(os.path.join(HERE, "golden.json")))
        pixel_sets(meta, PIXEL_SETS_R3, np.random.default_rng(20261017))
        with open(os.path.join(HERE, "golden.json"), "w") as f:
            json.dump(meta, f, indent=1)
        return
    if ("--mesh" in sys.argv or "--png" in sys.argv) and os.path.exists(os.path.join(HERE, "golden.json")):
        meta = json.load(open(os.path.join(HERE, "golden.json")))
        if "--png" in sys.argv:
            png_fixtures(meta)
        if "--mesh" in sys.argv:
            mesh_fixtures(meta)
        with open(os.path.join(HERE, "golden.json"), "w") as f:
            json.dump(meta, f, indent=1)
        return
    if not O.ref_available():
        subprocess.run([os.path.join(ROOT, "oracle", "ref", "build_ref.sh")], check=True)
    meta = {"generator": "tests/golden/gen_golden.py", "reference": "oracle/_ref/pt_ref (unmodified "
            "reference render.h/bvh.h/camera.h/image.h, g++ -O3)", "seed": 1, "images": {}, "pixels": {},
            "bvh": {}}
    rng = np.random.default_rng(20261015)
    for name, fac, res, spp, depth in IMAGES:
        sc = fac(res)
        img, m = O.ref_run(sc, spp, depth)
        np.save(os.path.join(HERE, name + ".npy"), img)
        meta["images"][name] = dict(scene=sc.name, scene_sha256=scene_hash(sc), res=list(res), spp=spp,
                                    depth=depth, ref_render_s=m["render_s"])
        print(name, img.shape, m["render_s"])
    pixel_sets(meta, PIXEL_SETS, rng)
    pixel_sets(meta, PIXEL_SETS_R3, np.random.default_rng(20261017))
    for name, fac in BVHS:
        sc = fac()
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "s.ptscene")
            with open(p, "w") as f:
                f.write(sc.to_ptscene())
            b = os.path.join(td, "bvh.bin")
            subprocess.run([O.REF_BIN, "--scene", p, "--spp", "1", "--depth", "1", "--res", "2", "2",
                            "--dump-bvh", b], check=True, capture_output=True)
            raw = open(b, "rb").read()
        nn, nt = np.frombuffer(raw[:8], dtype=np.int32)
        nodes = np.frombuffer(raw[8:8 + 40 * nn], dtype=O.NODE_DTYPE)
        idx = np.frombuffer(raw[8 + 40 * nn:], dtype=np.int32)
        assert idx.shape[0] == nt
        np.save(os.path.join(HERE, name + "_nodes.npy"), nodes)
        np.save(os.path.join(HERE, name + "_idx.npy"), idx)
        meta["bvh"][name] = dict(scene=sc.name, scene_sha256=scene_hash(sc), nodes=int(nn), tris=int(nt))
        print(name, nn, nt)
    png_fixtures(meta)
    # Known answers for the LCG (rng.h:14-20) from seed 1 — SURVEY.md §8(a) A9.
    meta["lcg_seed1"] = [1015568748, 1586005467, 2165703038, 3027450565]
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
