"""Coarse check against the reference's only published artefacts (SURVEY.md §4, §8(c)
acceptance): examples/*.png (README.md:23-46), 1024x1024, 10k spp, depth 5, rendered by
the reference's GLSL path. Their statistics are in tests/golden/ref_png_stats.json
(tests/golden/ref_png_stats.py). The framework renders the same seven scenes through
pt_ctx_render_rgb8 (gamma 2.2 + the CPU path's truncating quantisation, top row first)
and compares per-channel means and 8x8 block means.

Tolerances (fractions of 255), stated before the comparison and justified by what the
GLSL path does differently: its 8-bit output rounds to nearest
where save_png truncates (the GLSL image is brighter by ~0.5/255 = 0.002 on average), it
jitters rays over [w + 0.5, w + 1.5) instead of [w, w + 1) (a half-pixel shift: edges move
by half a pixel), and it uses another RNG (at 10k spp the per-pixel noise averages out in
a mean over 1M or 16k pixels). Means: |delta| <= 0.004 (one 8-bit step); block means over
128x128 pixels: |delta| <= 0.01 (a half-pixel edge shift in a 128-pixel block moves its mean
by at most 0.5/128 of the edge contrast, plus the rounding offset)."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT

MEAN_TOL = 0.004
BLOCK_TOL = 0.01


def _stats():
    with open(os.path.join(ROOT, "tests", "golden", "ref_png_stats.json")) as f:
        return json.load(f)


def test_reference_png_stats_fixture():
    st = _stats()
    assert set(st["images"]) == {"cornell", "mcornell_r0", "mcornell_r0.05", "mcornell_r0.1", "mcornell_r0.3",
                                 "mcornell_r0.5", "mcornell_r0.8"}
    for im in st["images"].values():
        assert im["shape"] == [1024, 1024] and len(im["blocks"]) == st["grid"]


@pytest.mark.gpu
def test_reference_png_statistics(tmp_path):
    import ptamd
    from ptamd import scenes
    st = _stats()
    g = st["grid"]
    r = ptamd.Renderer(0)
    report = {}
    try:
        for name, ref in st["images"].items():
            sc = scenes.cornell((1024, 1024)) if name == "cornell" else \
                scenes.modified_cornell(float(np.float32(float(name.split("_r")[1]))), (1024, 1024))
            r.set_scene(ptamd.BVH.from_scene(sc))
            rgb, _ = r.render_rgb8(ptamd.Camera.from_spec(sc.camera), 10000, 5, flip=True)
            x = rgb.astype(np.float64) / 255.0
            mean = x.mean(axis=(0, 1))
            blocks = x.reshape(g, 1024 // g, g, 1024 // g, 3).mean(axis=(1, 3))
            dm = mean - np.array(ref["mean"])
            db = blocks - np.array(ref["blocks"])
            report[name] = {"mean": mean.round(6).tolist(), "ref_mean": ref["mean"], "delta_mean": dm.round(6).tolist(),
                            "max_abs_delta_block": float(np.abs(db).max())}
    finally:
        r.close()
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "ref_png_compare.json"), "w") as f:
        json.dump(report, f, indent=1)
    for name, rep in report.items():
        assert max(abs(v) for v in rep["delta_mean"]) <= MEAN_TOL, (name, rep)
        assert rep["max_abs_delta_block"] <= BLOCK_TOL, (name, rep)
