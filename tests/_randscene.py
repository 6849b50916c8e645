"""Seeded random scenes for the parity tests (test infrastructure): tests/test_gpu_parity.py
renders them on every kernel path against the oracle, tests/test_oracle_golden.py checks the
oracle against the compiled reference on them."""
import numpy as np


def random_scene(seed, n_tris, res):
    """A seeded random scene: a closed room (12 triangles of the box [-10, 510]^3, so paths
    bounce) around `n_tris` random triangles, materials drawn from EMIT / DIFFUSE (random
    albedo, some with emission) / SPECULAR (random roughness), and a camera inside looking
    in a random direction. The room's walls do not emit. Every value is a float32."""
    from ptamd import scenes
    rng = np.random.default_rng(seed)
    f = lambda x: float(np.float32(x))  # noqa: E731
    def mat(emitters=True):
        k = rng.random()
        if emitters and k < 0.15:
            return scenes.Material.make(scenes.EMIT, 0, tuple(f(c) for c in rng.uniform(0.2, 4.0, 3)))
        if k < 0.7:
            emit = tuple(f(c) for c in rng.uniform(0, 0.5, 3)) if rng.random() < 0.2 else 0
            return scenes.Material.make(scenes.DIFFUSE, tuple(f(c) for c in rng.uniform(0, 1, 3)), emit)
        return scenes.Material.make(scenes.SPECULAR, tuple(f(c) for c in rng.uniform(0, 1, 3)), 0, f(rng.uniform(0, 1)))
    fwd = rng.normal(size=3)
    fwd[1] *= 0.3  # keep forward away from the up vector
    cam = scenes.CameraSpec(tuple(f(c) for c in rng.uniform(150, 350, 3)), tuple(f(c) for c in fwd / np.linalg.norm(fwd)),
                            (0.0, 1.0, 0.0), tuple(res), f(rng.uniform(40, 90)), 1.0)
    sc = scenes.Scene(f"random_{seed}_{n_tris}", cam)
    lo, hi = -10.0, 510.0
    c = [(x, y, z) for x in (lo, hi) for y in (lo, hi) for z in (lo, hi)]
    room = [(0, 1, 3), (0, 3, 2), (4, 6, 7), (4, 7, 5), (0, 4, 5), (0, 5, 1), (2, 3, 7), (2, 7, 6), (0, 2, 6), (0, 6, 4),
            (1, 5, 7), (1, 7, 3)]
    wall = mat(False)
    for a, b, d in room:
        sc.add([(c[a], c[b], c[d])], wall if rng.random() < 0.8 else mat(False))
    for _ in range(n_tris):
        p = rng.uniform(0, 500, 3)
        v = [tuple(f(x) for x in p + rng.normal(scale=rng.uniform(5, 80), size=3)) for _ in range(3)]
        sc.add([tuple(v)], mat())
    return sc
