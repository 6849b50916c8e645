"""gamma_correct + save_png quantisation (image.h:41-55, render.h:99-100).

The oracle (oracle_rgb8) is pinned to the reference's own PNG bytes (pt_ref --png,
tests/golden/*_png.npy). The host product path (pt_image_to_rgb8) and the device
quantiser's threshold table (pt_rgb8_thresholds, used by pt_ctx_render_rgb8) are
checked against the oracle: the table on every float of [-1, 2] for gamma 2.2 and on
every threshold's neighbourhood for other gammas. Bar: bit-exact (bytes).
"""
import numpy as np
import pytest

import _oracle as O
from conftest import load_golden

PNGS = ["cornell_64_s16_d5", "cornell_48x40_s8_d8", "mcornell_r0.3_64_s8_d5"]
GAMMAS = [2.2, 1.0, 0.5, 1.8, 2.4, 3.0, 0.25, 1 / 3]


@pytest.mark.parametrize("name", PNGS)
def test_oracle_rgb8_matches_reference_png(golden_meta, name):
    assert golden_meta["png"][name]["image"] == name
    assert np.array_equal(O.rgb8(load_golden(name)), load_golden(name + "_png"))


@pytest.mark.parametrize("name", PNGS)
def test_host_rgb8_matches_reference_png(name):
    import ptamd
    assert np.array_equal(ptamd.to_rgb8(load_golden(name)), load_golden(name + "_png"))


def _neighbourhood(thr):
    """Every threshold +-4 ulps, the special values and a random spread."""
    u = thr.view(np.uint32).astype(np.int64)
    near = (u[:, None] + np.arange(-4, 5)[None, :]).ravel()
    near = near[(near >= 0) & (near < 0x7F800000)].astype(np.uint32).view(np.float32)
    special = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-30, -1e-30, 0.5, -0.5, 1.0, -1.0, 2.0, -2.0, 1e30, -1e30,
                        np.inf, -np.inf, np.nan, -np.nan], np.float32)
    rnd = np.random.default_rng(11).uniform(-0.5, 2.5, 4096).astype(np.float32)
    return np.concatenate([near, -near, special, rnd])


def rule(x, thr, mode):
    """The device quantiser (pt_rgb8_kernel) restated in numpy."""
    x = np.asarray(x, np.float32)
    out = np.searchsorted(thr, np.abs(x), side="right").astype(np.uint8)
    neg = x < 0
    if mode != 2:
        out[neg] = 255 if mode == 0 else 0
    out[np.isnan(x)] = 255
    return out


@pytest.mark.parametrize("gamma", GAMMAS)
def test_threshold_table_on_neighbourhoods(gamma):
    import ptamd
    thr, mode = ptamd.rgb8_thresholds(gamma)
    assert np.all(np.diff(thr) >= 0) and thr[0] > 0
    x = _neighbourhood(thr)
    n = -(-x.size // 3)
    img = np.zeros(3 * n, np.float32)
    img[: x.size] = x
    want = O.rgb8(img.reshape(1, n, 3), gamma).reshape(-1)[: x.size]
    assert np.array_equal(rule(x, thr, mode), want)
    assert mode == (2 if gamma in (0.5, 0.25) else 1 if gamma in (1.0, 1 / 3) else 0)


def test_threshold_table_every_float_gamma22():
    """All 2^30 floats of [0, 1] and their negatives, and [1, 2] (powf >= 1 -> 255 above)."""
    import ptamd
    thr, mode = ptamd.rgb8_thresholds(2.2)
    sweep = lambda lo, hi: O.lib().oracle_rgb8_sweep(2.2, O._p(thr), mode, lo, hi, 1, 8)
    assert sweep(0x00000000, 0x3F800001) == 0
    assert sweep(0x80000000, 0xBF800001) == 0
    assert sweep(0x3F800001, 0x40000001) == 0
    assert O.lib().oracle_rgb8_sweep(2.2, O._p(thr), mode, 0x40000001, 0xFFFFFFFF, 4099, 8) == 0


@pytest.mark.parametrize("gamma", [0.0, -1.0, float("nan"), 1e-40])
def test_threshold_table_rejects_bad_gamma(gamma):
    import ptamd
    with pytest.raises(ptamd.PTError):
        ptamd.rgb8_thresholds(gamma)
