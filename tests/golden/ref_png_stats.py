#!/usr/bin/env python3
"""Statistics of the reference's published renders (examples/*.png, README.md:23-46):
per-channel means and an 8x8 grid of 128x128-pixel block means (fractions of 255) of
each 1024x1024 8-bit image, written to tests/golden/ref_png_stats.json. Run in the
container that holds /root/reference; the GPU test test_reference_png_statistics
compares the framework's renders of the same scenes with these numbers. The images
themselves come from the reference's GLSL path (another RNG, a half-pixel offset,
round-to-nearest 8-bit output), so they pin the converged image only coarsely.
usage: python tests/golden/ref_png_stats.py [/root/reference]
"""
import json
import os
import sys

import numpy as np
from PIL import Image

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
FILES = {"cornell": "cornell_box.png", "mcornell_r0": "mod0.png", "mcornell_r0.05": "mod0.05.png",
         "mcornell_r0.1": "mod0.1.png", "mcornell_r0.3": "mod0.3.png", "mcornell_r0.5": "mod0.5.png",
         "mcornell_r0.8": "mod0.8.png"}
GRID = 8


def stats(rgb: np.ndarray) -> dict:
    x = rgb.astype(np.float64) / 255.0
    H, W, _ = x.shape
    blocks = x.reshape(GRID, H // GRID, GRID, W // GRID, 3).mean(axis=(1, 3))
    return {"shape": [H, W], "mean": [round(float(v), 6) for v in x.mean(axis=(0, 1))],
            "blocks": np.round(blocks, 6).tolist()}


def main():
    out = {"source": "examples/*.png of the reference (GLSL render_gpu, 10k spp, depth 5; README.md:23-46)",
           "grid": GRID, "images": {}}
    for name, fn in FILES.items():
        img = np.asarray(Image.open(os.path.join(REF, "examples", fn)).convert("RGB"))
        out["images"][name] = {"file": fn, **stats(img)}
        print(name, out["images"][name]["mean"])
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_png_stats.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
