"""libm restatements used on the path (acosf, sincosf) against the host glibc,
and unit known-answer tests of the primitives (slab test, Möller–Trumbore,
BRDF draw order) through the oracle."""
import ctypes as C

import numpy as np
import pytest

import _oracle as O


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def test_acosf_sampled_vs_glibc():
    """Sampled check (the exhaustive one is test_libm_exhaustive_*)."""
    x = np.concatenate([np.linspace(-1, 1, 200001, dtype=np.float32),
                        np.random.default_rng(1).uniform(-1, 1, 200000).astype(np.float32)])
    got = np.empty_like(x)
    O.lib().oracle_acosf_n(_ptr(x), x.size, _ptr(got))
    libm = C.CDLL("libm.so.6")
    libm.acosf.argtypes = [C.c_float]
    libm.acosf.restype = C.c_float
    for i in range(0, x.size, 997):
        assert np.float32(libm.acosf(float(x[i]))).view(np.uint32) == got[i].view(np.uint32), x[i]


@pytest.mark.parametrize("which,lo,hi", [(0, -1.0, 1.0), (1, -2.0, 7.0)])
def test_libm_exhaustive(which, lo, hi):
    """Every float in the path's domain: acosf over [-1, 1] (argument 2u-1), sincosf over
    [-2, 7] (theta in [-pi/2, pi/2], phi in [0, 2pi]). ~15 s each."""
    tested = C.c_uint64(0)
    bad = O.lib().oracle_libm_sweep(which, C.c_float(lo), C.c_float(hi), C.byref(tested))
    assert tested.value > 2_000_000_000
    assert bad == 0


def _tri(v, o, d):
    v = np.asarray(v, np.float32)
    o = np.asarray(o, np.float32)
    d = np.asarray(d, np.float32)
    t = C.c_float(0)
    hit = O.lib().oracle_tri_hit(_ptr(v), _ptr(o), _ptr(d), C.byref(t))
    return hit, t.value


def test_moller_trumbore_known_answers():
    tri = [0, 0, 0, 1, 0, 0, 0, 1, 0]
    assert _tri(tri, [0.25, 0.25, 1], [0, 0, -1]) == (1, 1.0)
    assert _tri(tri, [0.25, 0.25, 1], [0, 0, 1])[0] == 0      # behind: t < 0
    assert _tri(tri, [0.6, 0.6, 1], [0, 0, -1])[0] == 0       # u + v > 1
    assert _tri(tri, [0.5, 0.5, 1], [0, 0, -1])[0] == 1       # on the diagonal edge: u + v == 1 accepted
    assert _tri(tri, [0.0, 0.0, 1], [0, 0, -1])[0] == 1       # at a vertex
    assert _tri(tri, [0.25, 0.25, 1], [1, 0, 0])[0] == 0      # parallel: |a| < EPS


def test_moller_trumbore_eps_is_compared_in_double():
    """|a| < 1e-6 with EPS a double (linalg.h:11, triangle.h:31): a == 1e-6f (just below the
    double 1e-6) is rejected, the next float up is accepted."""
    below = np.float32(1e-6)          # 0x358637BD = 9.99999997e-07 < 1e-6
    above = np.nextafter(below, np.float32(1))
    assert float(below) < 1e-6 < float(above)
    # triangle in the z=0 plane with e1 = (1,0,0), e2 = (0,1,0); a = e1 . (d x e2) = -d.z
    for dz, expect in ((below, 0), (above, 1)):
        hit, _ = _tri([0, 0, 0, 1, 0, 0, 0, 1, 0], [0.25, 0.25, 1], [0, 0, -dz])
        assert hit == expect, dz


def test_slab_semantics_with_nan():
    def slab(lb, rt, o, inv):
        f = lambda v: np.asarray(v, np.float32)
        return O.lib().oracle_slab(_ptr(f(lb)), _ptr(f(rt)), _ptr(f(o)), _ptr(f(inv)))
    assert slab([0, 0, 0], [1, 1, 1], [0.5, 0.5, -1], [np.inf, np.inf, 1]) == 1
    assert slab([0, 0, 0], [1, 1, 1], [0.5, 0.5, 2], [np.inf, np.inf, 1]) == 0   # box behind: tmax < 0
    # Origin on a slab plane with a zero direction component: 0 * inf = NaN. std::max/min
    # return the first operand when a compare involves NaN and min_element/max_element
    # start from the x slab, so a NaN x slab poisons tmin/tmax -> miss (IEEE maxNum
    # would ignore the NaN and report a hit) ...
    assert slab([0, 0, 0], [1, 1, 1], [0.0, 0.5, -1], [np.inf, np.inf, 1]) == 0
    # ... while a NaN in the z slab is skipped by the scan -> hit.
    assert slab([0, 0, 0], [1, 1, 1], [0.5, 0.5, 0.0], [1, 1, np.inf]) == 1
    assert slab([0, 0, 0], [1, 1, 1], [1.5, 0.5, -1], [np.inf, np.inf, 1]) == 0


def test_brdf_draw_order():
    """Diffuse: u then v. Specular: z, y, x per jitter (g++ evaluates vec3(...) args right
    to left). The state after the call = number of draws."""
    d = np.array([0, 0, -1], np.float32)
    n = np.array([0, 0, 1], np.float32)
    out = np.zeros(3, np.float32)
    a, c = 1664525, 1013904223
    step = lambda s, k: [s := (a * s + c) % 2 ** 32 for _ in range(k)][-1]
    s_after = O.lib().oracle_brdf(12345, 2, C.c_float(0), _ptr(d), _ptr(n), _ptr(out))
    assert s_after == step(12345, 2)
    assert float(np.dot(out, n)) >= 0
    s_after = O.lib().oracle_brdf(777, 3, C.c_float(0.0), _ptr(d), _ptr(n), _ptr(out))
    assert s_after == step(777, 3)  # roughness 0: one rejection round
    np.testing.assert_array_equal(out, np.array([0, 0, 1], np.float32))
    # roughness 0.3: jitter x comes from the THIRD draw
    st = 99
    s1 = step(st, 1); s2 = step(st, 2); s3 = step(st, 3)
    r = lambda s: np.float32(np.float32(s) / np.float32(2 ** 32))
    jx, jy, jz = [(r(v) - np.float32(0.5)) * np.float32(0.3) for v in (s3, s2, s1)]
    O.lib().oracle_brdf(st, 3, C.c_float(0.3), _ptr(d), _ptr(n), _ptr(out))
    ret = np.array([0 + jx, 0 + jy, 1 + jz], np.float32)
    if ret[2] >= 0:
        exp = ret / np.float32(np.sqrt(np.float32(np.dot(ret, ret))))
        np.testing.assert_allclose(out, exp, rtol=1e-6)


def test_theta_table_index_covers_every_lcg_draw():
    """The device's theta table (pt_math.h: hemisphere_dir_tab) holds (sin, cos) of
    theta = acosf(x) - M_PI_2 for the 2^25 + 1 grid points x = k 2^-24 of [-1, 1]. That covers
    the path exactly when x = 2 rand01 - 1 (material.h:8-9) lies on the grid for EVERY 32-bit
    LCG output: checked here for all 2^32 of them (x = 1 is reached by 128)."""
    import ctypes as C
    one = C.c_uint64(0)
    assert O.lib().oracle_theta_grid_check(C.byref(one)) == 0
    assert one.value == 128
