"""The console contract of the drop-in render_cpu / render_gpu (Python host layer):
the reference's lines (render.h:79-101 and 127-149) byte for byte but for the timings,
and the PNG they write decodes to the gamma-corrected, quantised image."""
import re

import numpy as np
import pytest


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["cpu", "gpu"])
def test_python_render_console_and_png(tmp_path, capfd, which):
    from PIL import Image as PILImage
    import ptamd
    from ptamd import scenes
    sc = scenes.cornell((40, 24))
    cam = ptamd.Camera.from_spec(sc.camera)
    fn = str(tmp_path / "o.png")
    if which == "cpu":
        assert ptamd.render_cpu(cam, ptamd.BVH.from_scene(sc), 8, 5, fn)
        want = ("Rendered: 0/24 rows." + "".join(f"\rRendered: {k}/24 rows." for k in range(1, 25)) +
                "\nDone in T seconds.\nColor correcting...\nSaved to " + fn + "\n")
    else:
        assert ptamd.render_gpu(cam, ptamd.BVH.from_scene(sc), 8, 5, (16, 16), fn)
        want = ("Rendered: 0/6 chunks." + "".join(f"\rRendered: {k}/6 chunks." for k in range(1, 7)) +
                "\nDone in T seconds.\nSaved to " + fn + "\n")
    got = re.sub(r"Done in \d+\.\d\d seconds", "Done in T seconds", capfd.readouterr().out)
    if got != want:
        i = next((k for k in range(min(len(got), len(want))) if got[k] != want[k]), min(len(got), len(want)))
        raise AssertionError(f"stdout differs at {i}: got {got[max(0, i - 40):i + 80]!r} want {want[max(0, i - 40):i + 80]!r}")
    img, _ = ptamd.render(cam, ptamd.BVH.from_scene(sc), 8, 5)
    assert np.array_equal(np.asarray(PILImage.open(fn).convert("RGB")), ptamd.to_rgb8(img))


@pytest.mark.gpu
def test_progress_reports_monotone_to_total():
    """pt_params.progress over several launches and several parts (one device listed
    twice): done increases to total = W * H * spp, one report at a time."""
    import ptamd
    from ptamd import scenes
    sc = scenes.cornell((64, 48))
    seen = []
    img, st = ptamd.render_rgb8(ptamd.Camera.from_spec(sc.camera), ptamd.BVH.from_scene(sc), 40, 5, [0, 0],
                                batch_spp=8, progress=lambda d, t: seen.append((d, t)))
    assert st["trace_launches"] >= 2 * 5
    assert seen and all(t == 64 * 48 * 40 for _, t in seen)
    assert [d for d, _ in seen] == sorted(set(d for d, _ in seen)) and seen[-1][0] == 64 * 48 * 40
