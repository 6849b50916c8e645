"""GPU parity: the gfx950 trace kernel (through the C ABI) against the reference.

Bar: bit-exact. Every render here must equal the reference's own output for
the same per-sample seeds (golden fixtures from oracle/_ref/pt_ref) or the CPU
oracle (pinned to those fixtures by test_oracle_golden.py) bit for bit, with
the same ray count.
"""
import numpy as np
import pytest

from conftest import load_golden, scene_for, scene_hash

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ptamd_mod():
    import ptamd
    if ptamd.lib().pt_device_count() <= 0:
        pytest.fail("no HIP device visible: the gpu tests must run on the GPU box")
    return ptamd


def _render(ptamd, scene, spp, depth, **kw):
    bvh = ptamd.BVH.from_scene(scene)
    cam = ptamd.Camera.from_spec(scene.camera)
    return ptamd.render(cam, bvh, spp, depth, **kw)


def _bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def test_golden_images_bitexact(ptamd_mod, golden_meta):
    import _oracle as O
    for name, m in golden_meta["images"].items():
        sc = scene_for(m["scene"], m["res"])
        assert scene_hash(sc) == m["scene_sha256"], name
        img, st = _render(ptamd_mod, sc, m["spp"], m["depth"])
        ref = load_golden(name)
        diff = np.abs(img - ref)
        assert _bits_equal(img, ref), f"{name}: {int((img.view(np.uint32) != ref.view(np.uint32)).sum())} " \
                                      f"words differ, max abs {diff.max()}"
        if m["res"][0] * m["res"][1] * m["spp"] <= 70000:
            _, rays = O.render(sc, m["spp"], m["depth"])
            assert st["rays"] == rays, name
        assert st["paths"] == m["res"][0] * m["res"][1] * m["spp"]


def test_full_size_sampled_pixels(ptamd_mod, golden_meta, monkeypatch):
    """Configs 2-5 at full resolution and spp: EVERY pinned pixel is bit-exact (64 of
    config 2, 12 + 8 + 4 x 8 of config 3 (all six roughness values), 20 of config 4 incl.
    the on-sphere ones, 8 of config 5), on the kernel bench.py times: the scene's hipRTC
    flat kernel (compile waited for, kernel_path 3) for configs 2, 3 and 5, the 8-wide walk
    (kernel_path 4) for config 4. Renders each distinct row holding pinned pixels once (row
    partition with band 1). Then the first pinned row of every flat config again on the
    table kernels a cold process runs while its scene kernel compiles (PT_RTC=0: the box table
    in kernel arguments, with the scene's flags, kernel_path 5, and fully generic, 2)."""
    checked = 0
    flat_rows = []
    for name, m in golden_meta["pixels"].items():
        sc = scene_for(m["scene"], m["res"])
        W, H = m["res"]
        ref = load_golden(name)
        assert ref.shape == (len(m["pixels"]), 3), name
        bvh = ptamd_mod.BVH.from_scene(sc)
        cam = ptamd_mod.Camera.from_spec(sc.camera)
        r = ptamd_mod.Renderer(0)
        r.set_scene(bvh)
        r.prepare()  # the timed (hipRTC) kernel from the first launch on
        want_path = 4 if m["scene"].startswith("sphere") else 3
        by_row = {}
        for i, (w, h) in enumerate(m["pixels"]):
            by_row.setdefault(h, []).append((i, w))
        for h, cols in sorted(by_row.items()):
            # one-row part: part_count = H, band 1 -> part h is exactly row h
            img, st = r.render(cam, m["spp"], m["depth"], part_index=h, part_count=H, band_rows=1)
            assert img.shape == (1, W, 3)
            assert st["kernel_path"] == want_path, (name, st["kernel_path"])
            for i, w in cols:
                assert _bits_equal(img[0, w], ref[i]), f"{name} pixel {(w, h)}: {img[0, w]} vs {ref[i]}"
                checked += 1
        r.close()
        if want_path == 3:
            h, cols = sorted(by_row.items())[0]
            flat_rows.append((name, m, bvh, cam, ref, h, cols))
    assert checked == sum(len(m["pixels"]) for m in golden_meta["pixels"].values())
    # the table kernels a cold frame runs while the scene kernel compiles: with the scene's
    # flags baked in (path 5, every BASELINE flat scene qualifies) and fully generic (path 2)
    monkeypatch.setenv("PT_RTC", "0")
    for fast, want in (("1", 5), ("0", 2)):
        monkeypatch.setenv("PT_FLAT_FAST", fast)
        for name, m, bvh, cam, ref, h, cols in flat_rows:
            r = ptamd_mod.Renderer(0)
            r.set_scene(bvh)
            img, st = r.render(cam, m["spp"], m["depth"], part_index=h, part_count=m["res"][1], band_rows=1)
            assert st["kernel_path"] == want, (name, st["kernel_path"])
            for i, w in cols:
                assert _bits_equal(img[0, w], ref[i]), f"{name} table kernel {want}, pixel {(w, h)}"
            r.close()


@pytest.mark.parametrize("kind", ["flat", "wide"])
def test_work_pool_refill_sizes_bitexact(ptamd_mod, monkeypatch, kind):
    """Launches large enough for full-size refills of the work pool (claim_work, pt_trace.h):
    the default refill size (items / (waves x 64), here 256 or 341 items), ~4 refills per wave
    (PT_POOL_REFILLS=4: 1024 items) and no static first pools (PT_STATIC_MODE=0) give the same
    image bit for bit with the same ray and path counts; and rows of it equal the same rows
    rendered alone (one-row launches of 64-item refills: the oracle-checked configuration of
    test_full_size_sampled_pixels)."""
    from ptamd import scenes
    if kind == "wide":
        monkeypatch.setenv("PT_WIDE", "1")
        sc = scenes.sphere_in_cornell(24, (1024, 1024))
    else:
        sc = scenes.cornell((1024, 1024))
    bvh = ptamd_mod.BVH.from_scene(sc)
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    keys = ("PT_POOL_REFILLS", "PT_STATIC_MODE")
    r = ptamd_mod.Renderer(0)
    try:
        r.set_scene(bvh)
        r.prepare()
        out = {}
        for name, env in (("default", {}), ("refills4", {"PT_POOL_REFILLS": "4"}), ("nostatic", {"PT_STATIC_MODE": "0"})):
            for k in keys:
                monkeypatch.delenv(k, raising=False)
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            out[name] = r.render(cam, 256, 4, batch_spp=128)  # two launches of 134M samples
        img, st = out["default"]
        assert st["paths"] == 1024 * 1024 * 256 and st["trace_launches"] == 2
        for name in ("refills4", "nostatic"):
            assert _bits_equal(out[name][0], img), name
            assert out[name][1]["rays"] == st["rays"] and out[name][1]["paths"] == st["paths"], name
        for k in keys:
            monkeypatch.delenv(k, raising=False)
        for h in (0, 137, 1023):
            row, _ = r.render(cam, 256, 4, part_index=h, part_count=1024, band_rows=1)
            assert _bits_equal(row[0], img[h]), h
    finally:
        r.close()


@pytest.mark.parametrize("scene_name,res,spp,depth", [
    ("cornell", (37, 29), 7, 4),
    ("cornell", (64, 48), 3, 8),
    ("modified_cornell_r0.5", (40, 40), 6, 5),
    ("modified_cornell_r0.05", (32, 24), 5, 6),
    ("modified_cornell_r0.1", (16, 16), 9, 3),
    ("tri3", (50, 50), 11, 5),
])
def test_vs_oracle_bitexact(ptamd_mod, scene_name, res, spp, depth):
    import _oracle as O
    sc = scene_for(scene_name, res)
    img, st = _render(ptamd_mod, sc, spp, depth)
    ref, rays = O.render(sc, spp, depth)
    assert _bits_equal(img, ref), f"max abs {np.abs(img - ref).max()}"
    assert st["rays"] == rays
    assert st["paths"] == res[0] * res[1] * spp


def test_partition_and_batching_invariance(ptamd_mod):
    """Any row partition, batch size or work-item size gives the same bits."""
    from ptamd import scenes
    sc = scenes.cornell((48, 45))
    full, st_full = _render(ptamd_mod, sc, 12, 5)
    bvh = ptamd_mod.BVH.from_scene(sc)
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    r = ptamd_mod.Renderer(0)
    r.set_scene(bvh)
    for parts, band in [(2, 8), (3, 4), (5, 1), (8, 16)]:
        rays = 0
        rows_seen = []
        for p in range(parts):
            img, st = r.render(cam, 12, 5, part_index=p, part_count=parts, band_rows=band)
            rows = [h for h in range(45) if (h // band) % parts == p]
            rows_seen += rows
            assert _bits_equal(img, full[rows]), (parts, band, p)
            rays += st["rays"]
        assert sorted(rows_seen) == list(range(45))
        assert rays == st_full["rays"]
    for batch, per_item in [(1, 1), (5, 2), (12, 12), (7, 3)]:
        img, st = r.render(cam, 12, 5, batch_spp=batch, samples_per_item=per_item)
        assert _bits_equal(img, full), (batch, per_item)
        assert st["rays"] == st_full["rays"]
    r.close()


def _launches(spp, batch, tail_div):
    """Trace launches of a frame of `spp` samples in batches of `batch` with the fused
    accumulation's tail batch (render_range: batch_at)."""
    tail = max(1, batch // tail_div) if spp > batch and tail_div > 0 else 0
    s = n = 0
    while s < spp:
        left = spp - s
        s += min(batch, left) if tail <= 0 or left <= tail else (left - tail if left <= batch + tail else batch)
        n += 1
    return n


def test_multi_batch_frames_bitexact(ptamd_mod, monkeypatch):
    """Frames of several sample batches (one launch each, accumulate passes in sample
    order) give the golden bits and ray count for any batch size, on the flat and the
    wide kernel, and across progressive frames of several batches."""
    import _oracle as O
    from ptamd import scenes
    sc = scenes.cornell((48, 45))
    full, st_full = _render(ptamd_mod, sc, 12, 5, batch_spp=12)
    bvh = ptamd_mod.BVH.from_scene(sc)
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    # the fused accumulation's tail batch (PT_TAIL_DIV: the last batch is batch / div samples)
    for div in (0, 2, 4):
        monkeypatch.setenv("PT_TAIL_DIV", str(div))
        r = ptamd_mod.Renderer(0)
        r.set_scene(bvh)
        for batch in (1, 2, 5, 6, 11):
            img, st = r.render(cam, 12, 5, batch_spp=batch)
            assert _bits_equal(img, full), (div, batch)
            assert st["rays"] == st_full["rays"] and st["trace_launches"] == _launches(12, batch, div), (div, batch)
        for s_first, k in ((0, 3), (3, 4), (7, 5)):  # progressive frames of several batches each
            img, _ = r.render_progressive(cam, s_first, k, 5, batch_spp=2)
        assert _bits_equal(img, full), div
        r.close()
    monkeypatch.delenv("PT_TAIL_DIV")
    # the previous batch summed inside the next launch (fused accumulation, default) or by a
    # separate pass after every launch, on the hipRTC kernel, the wide walk and the tree walk
    paths = {"PT_RTC_WAIT": (3,), "PT_FLAT": (4,), "PT_WIDE": (0, 1)}
    for env in ({"PT_RTC_WAIT": "1"}, {"PT_RTC_WAIT": "1", "PT_FUSED_ACC": "0"}, {"PT_FLAT": "0"},
                {"PT_FLAT": "0", "PT_WIDE": "0"}):
        with monkeypatch.context() as m:
            for k, v in env.items():
                m.setenv(k, v)
            r = ptamd_mod.Renderer(0)
            r.set_scene(bvh)
            for batch in (1, 3, 5):
                img, st = r.render(cam, 12, 5, batch_spp=batch)
                assert _bits_equal(img, full), (env, batch)
                assert st["rays"] == st_full["rays"]
                assert st["kernel_path"] in paths[[k for k in paths if k in env][-1]], env
            for s_first, k in ((0, 5), (5, 7)):
                img, _ = r.render_progressive(cam, s_first, k, 5, batch_spp=2)
            assert _bits_equal(img, full), env
            r.close()
    monkeypatch.setenv("PT_WIDE", "1")
    sc = scenes.sphere_in_cornell(32, (40, 32))
    ref, rays = O.render(sc, 6, 5)
    img, st = _render(ptamd_mod, sc, 6, 5, batch_spp=2)
    assert _bits_equal(img, ref) and st["rays"] == rays


@pytest.mark.parametrize("env", [{"PT_RTC": "0"}, {"PT_RTC": "0", "PT_FLAT_FAST": "0"}, {"PT_FLAT": "0"}])
def test_generic_kernels_bitexact(ptamd_mod, monkeypatch, env):
    """The flat table kernels (kernel-argument box table, PT_RTC=0: with the scene's flags baked
    in, round 6, or fully generic with PT_FLAT_FAST=0) and the tree walk (PT_FLAT=0) give the
    reference's bits too (default: hipRTC-specialised flat kernel)."""
    import _oracle as O
    from ptamd import scenes
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for sc, spp, depth in [(scenes.cornell((40, 33)), 5, 5), (scenes.modified_cornell(0.3, (32, 32)), 4, 5)]:
        img, st = _render(ptamd_mod, sc, spp, depth)
        ref, rays = O.render(sc, spp, depth)
        assert _bits_equal(img, ref) and st["rays"] == rays, (env, sc.name)
        if "PT_RTC" in env:
            assert st["kernel_path"] == (2 if env.get("PT_FLAT_FAST") == "0" else 5), (env, sc.name)


@pytest.mark.parametrize("planes", ["byte", "f16", "f32"])
@pytest.mark.parametrize("width,top,nb,umat,single,compact",
                         [("4", "0", "1", "64", "1", "1"), ("8", "0", "1", "64", "1", "1"),
                          ("8", "0", "0", "64", "0", "1"), ("8", "8192", "1", "64", "1", "1"),
                          ("4", "65536", "0", "64", "0", "1"), ("8", "0", "1", "0", "1", "1"),
                          ("4", "0", "1", "0", "0", "1"), ("8", "0", "1", "64", "0", "1"),
                          ("8", "0", "1", "64", "1", "0"), ("8", "0", "0", "64", "0", "0")])
def test_wide_tree_bitexact(ptamd_mod, monkeypatch, width, top, nb, umat, single, compact, planes):
    """The wide-tree walk (default for scenes past the flat list, e.g. config 4's mesh),
    forced onto small scenes with PT_WIDE=1 and on a 2k-triangle sphere mesh, against
    the oracle: same bits, same ray count; with and without the top levels in LDS, with
    the branch-free (tri_hit_nb, default) and the branchy triangle test in the drains,
    with the distinct-material table in LDS (default) and in global memory (umat 0), with
    the single-triangle-leaf queue entries (default for BVH::build trees) and the general
    leaf-range decode (single 0); child planes as quantised bytes, binary16 integers and
    the reference's own floats (PT_WIDE_PLANES, round 6); 48-B triangle records (compact 1, default for single-triangle leaves: edges
    and leaf box formed in the kernel) and the 64-B records (compact 0)."""
    import _oracle as O
    from ptamd import scenes
    monkeypatch.setenv("PT_WIDE", "1")
    monkeypatch.setenv("PT_WIDE_PLANES", planes)
    monkeypatch.setenv("PT_WIDE_W", width)
    monkeypatch.setenv("PT_WIDE_TOP_BYTES", top)
    monkeypatch.setenv("PT_WIDE_NB", nb)
    monkeypatch.setenv("PT_UMAT_LDS_MAX", umat)
    monkeypatch.setenv("PT_WIDE_SINGLE", single)
    monkeypatch.setenv("PT_WIDE_COMPACT", compact)
    base = scenes.cornell((33, 33))
    axis_cam = scenes.CameraSpec((278.0, 274.4, 0.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0), (33, 33), 1e-3, 1.0)
    cases = [(scenes.cornell((40, 33)), 5, 5), (scenes.modified_cornell(0.3, (32, 32)), 4, 5),
             (scenes.sphere_in_cornell(32, (48, 40)), 4, 5),
             (scenes.Scene("axis", axis_cam, list(base.tris), list(base.mats)), 3, 5)]  # huge inv components
    for sc, spp, depth in cases:
        img, st = _render(ptamd_mod, sc, spp, depth)
        ref, rays = O.render(sc, spp, depth)
        assert st["kernel_path"] == 4, sc.name
        assert _bits_equal(img, ref) and st["rays"] == rays, (width, sc.name)


def test_wide_tree_with_caller_leaf_boxes_bitexact(ptamd_mod, monkeypatch):
    """A tree whose leaf boxes are not the triangles' AABBs (shrunk inside them, as a
    caller's own builder could hand over through the C ABI): the wide walk keeps the stored
    leaf boxes (64-B records) and matches the oracle walking the same nodes, bits and ray
    count (the 48-B records would rebuild the AABB and count extra hits)."""
    import _oracle as O
    from ptamd import scenes
    from test_capi import shrink_leaf_boxes
    monkeypatch.setenv("PT_WIDE", "1")
    sc = scenes.sphere_in_cornell(32, (48, 40))
    bvh = ptamd_mod.BVH.from_scene(sc)
    bvh.build()
    nodes = bvh.nodes.copy()
    assert shrink_leaf_boxes(nodes, bvh.tri_idx, bvh.verts()) > 0
    bvh.nodes = nodes
    assert ptamd_mod.scene_info(bvh)["wide_record_bytes"] == 64
    img, st = ptamd_mod.render(ptamd_mod.Camera.from_spec(sc.camera), bvh, 4, 5)
    ref, rays = O.render(sc, 4, 5, nodes=nodes, idx=bvh.tri_idx)
    assert st["kernel_path"] == 4
    assert _bits_equal(img, ref) and st["rays"] == rays


@pytest.mark.parametrize("lanes", ["64", "0"])
def test_theta_table_bitexact(ptamd_mod, monkeypatch, lanes):
    """hemisphere_sample's theta terms from the device table (pt_math.h: hemisphere_dir_tab):
    forced on every wave (PT_THETA_LANES=64) or off (0) in an all-diffuse scene on the flat
    (hipRTC) and wide kernels and in a specular scene, where the default (32) mixes table
    and computed waves; the oracle's bits and ray count either way."""
    import _oracle as O
    from ptamd import scenes
    monkeypatch.setenv("PT_THETA_LANES", lanes)
    for sc, spp, env in [(scenes.cornell((40, 36)), 6, {}), (scenes.modified_cornell(0.5, (36, 32)), 5, {}),
                         (scenes.sphere_in_cornell(32, (40, 32)), 4, {"PT_WIDE": "1"})]:
        with monkeypatch.context() as m:
            for k, v in env.items():
                m.setenv(k, v)
            img, st = _render(ptamd_mod, sc, spp, 5)
        ref, rays = O.render(sc, spp, 5)
        assert _bits_equal(img, ref) and st["rays"] == rays, (lanes, sc.name)


def _bits_equal_nan(a, b):
    """Bit equality, except that any two NaNs count as equal: x86 makes inf * 0 the negative
    default NaN and gfx950 the positive one (the payload is not part of the reference's
    arithmetic, its NaN-ness is)."""
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


@pytest.mark.parametrize("case,x2", [("default", True), ("hook_off", False), ("emit_2^50", True),
                                     ("emit_2^100", False), ("emit_2^126", False), ("albedo_2^127", False),
                                     ("albedo_subnormal", True)])
@pytest.mark.parametrize("depth", [5, 8])
def test_albedo_x2_unwinding_bitexact(ptamd_mod, monkeypatch, case, x2, depth):
    """The hipRTC flat kernel's unwinding with pre-doubled albedo (L * 2a instead of
    (2L) * a; enabled by the host's radiance bound, pt_kernel.hip: albedo_x2_ok) and without
    it: the oracle's bits and ray count at depth 5 (records loaded up front) and 8 (the
    per-level loop), with large emission (2^50: still enabled; 2^100: bound fails, off;
    2^126: the reference's 2L overflows to inf where L * 2a would not), an albedo of 2^127
    (2a = inf: a missed path's 0 * 2a would be NaN where the reference's (2 * 0) * a is 0)
    and a subnormal albedo (products in the subnormal range). The context's flag is the one
    the render uses (the gate was evaluated after the materials were dropped)."""
    import _oracle as O
    from ptamd import scenes
    sc = scenes.cornell((40, 36))
    for i, m in enumerate(sc.mats):
        if case.startswith("emit_") and m.type == scenes.EMIT:
            e = 2.0 ** int(case[7:])
            sc.mats[i] = scenes.Material(m.type, m.color, (e, e / 3, e / 7), m.roughness)
        if case == "albedo_subnormal" and m.type == scenes.DIFFUSE:
            sc.mats[i] = scenes.Material(m.type, tuple(c * 2.0 ** -140 for c in m.color), m.emit, m.roughness)
    if case == "albedo_2^127":
        m = sc.mats[0]
        assert m.type == scenes.DIFFUSE
        sc.mats[0] = scenes.Material(m.type, (2.0 ** 127, 1.5 * 2.0 ** 127, 2.0 ** 127), m.emit, m.roughness)
    bvh = ptamd_mod.BVH.from_scene(sc)
    if case == "hook_off":
        monkeypatch.setenv("PT_ALBEDO_X2", "0")
    monkeypatch.setenv("PT_RTC_WAIT", "1")
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    r = ptamd_mod.Renderer(0)
    try:
        r.set_scene(bvh)
        assert r.flags()["albedo_x2"] == x2 and r.flags()["rtc"]
        img, st = r.render(cam, 5, depth)
    finally:
        r.close()
    ref, rays = O.render(sc, 5, depth)
    assert st["kernel_path"] == 3
    if case == "albedo_2^127":
        assert np.isinf(ref).any()  # the case reaches the overflow it is meant to test
    assert _bits_equal_nan(img, ref) and st["rays"] == rays, case


@pytest.mark.parametrize("case,dark", [("default", True), ("hook_off", False), ("diffuse_emits", False),
                                       ("diffuse_emits_minus0", False), ("albedo_inf", False),
                                       ("specular_r0.8", True), ("specular_r2", False)])
def test_dark_path_skip_bitexact(ptamd_mod, monkeypatch, case, dark):
    """finish_path skips the unwinding of paths whose end value is +0 when every bounce
    material is dark (emission bits 0, finite albedo; PT_DARK_SKIP): the oracle's bits and ray
    counts on the hipRTC flat kernel, the generic flat kernel and the wide walk, with the skip
    on (Cornell), forced off (PT_DARK=0), and off because a diffuse wall emits (0.25, 0, 0), has
    emission -0 (+0 + (L a) c would give +0 where the reference keeps -0 only through the
    unwinding) or an infinite albedo (0 * inf is NaN); a specular room is dark at roughness 0.8
    and not at 2.0, where refl + j can cancel and cos theta be NaN (round 6, scene_dark)."""
    import _oracle as O
    from ptamd import scenes
    sc = scenes.cornell((36, 30))
    if case.startswith("specular_r"):
        sc = scenes.modified_cornell(float(case[len("specular_r"):]), (36, 30))
    m = sc.mats[0]
    assert m.type == scenes.DIFFUSE or case.startswith("specular_r")
    if case == "diffuse_emits":
        sc.mats[0] = scenes.Material(m.type, m.color, (0.25, 0.0, 0.0), m.roughness)
    elif case == "diffuse_emits_minus0":
        sc.mats[0] = scenes.Material(m.type, m.color, (-0.0, 0.0, 0.0), m.roughness)
    elif case == "albedo_inf":
        sc.mats[0] = scenes.Material(m.type, (float("inf"), 0.5, 0.5), m.emit, m.roughness)
    if case == "hook_off":
        monkeypatch.setenv("PT_DARK", "0")
    monkeypatch.setenv("PT_RTC_WAIT", "1")
    bvh = ptamd_mod.BVH.from_scene(sc)
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    ref, rays = O.render(sc, 5, 5)
    for env, path in (({}, 3), ({"PT_RTC": "0"}, 5 if dark else 2), ({"PT_WIDE": "1"}, 4)):
        with monkeypatch.context() as mp:
            for k, v in env.items():
                mp.setenv(k, v)
            r = ptamd_mod.Renderer(0)
            try:
                r.set_scene(bvh)
                assert r.flags()["dark"] == dark
                img, st = r.render(cam, 5, 5)
            finally:
                r.close()
        assert st["kernel_path"] == path, (case, env)
        assert _bits_equal_nan(img, ref) and st["rays"] == rays, (case, env)


@pytest.mark.parametrize("layout", ["", "0", "1"])
def test_flagged_slab_across_scenes_and_batches_bitexact(ptamd_mod, monkeypatch, layout):
    """Flagged slabs (TraceArgs::flags, dark scenes): only paths that do not end dark store a
    record and set its bit, and the accumulation adds only flagged records. One context renders
    a dark scene in several batches (fused and separate accumulation passes, a tail batch),
    then a scene that is not dark (dense slab), then the dark scene again, a specular dark
    scene, with progressive frames in between — on the flat and the wide kernel, and with the
    flags forced off (PT_FLAGS=0): every image is the oracle's. With the library's choice of
    bit layout (pixel-major for frames of several launches, sample-major for one) and with
    either layout forced for every frame (PT_FLAGS_PM)."""
    import _oracle as O
    from ptamd import scenes
    if layout:
        monkeypatch.setenv("PT_FLAGS_PM", layout)
    dark = scenes.cornell((40, 33))
    lit = scenes.cornell((40, 33))
    m = lit.mats[0]
    lit.mats[0] = scenes.Material(m.type, m.color, (0.125, 0.0, 0.25), m.roughness)
    spec = scenes.modified_cornell(0.3, (36, 30))
    refs = {id(sc): O.render(sc, 9, 5) for sc in (dark, lit, spec)}
    for env in ({}, {"PT_FUSED_ACC": "0"}, {"PT_WIDE": "1"}, {"PT_TAIL_DIV": "4"}, {"PT_FLAGS": "0"}):
        with monkeypatch.context() as mp:
            for k, v in env.items():
                mp.setenv(k, v)
            r = ptamd_mod.Renderer(0)
            try:
                for sc, batch in ((dark, 2), (lit, 4), (dark, 3), (spec, 2), (dark, 0), (lit, 0), (spec, 0), (dark, 2)):
                    bvh = ptamd_mod.BVH.from_scene(sc)
                    r.set_scene(bvh)
                    assert r.flags()["dark"] == (sc is not lit)
                    cam = ptamd_mod.Camera.from_spec(sc.camera)
                    img, st = r.render(cam, 9, 5, batch_spp=batch)
                    ref, rays = refs[id(sc)]
                    assert _bits_equal(img, ref) and st["rays"] == rays, (env, sc.name, batch)
                    for s_first, k in ((0, 4), (4, 5)):
                        img, _ = r.render_progressive(cam, s_first, k, 5, batch_spp=2)
                    assert _bits_equal(img, ref), (env, sc.name, "progressive")
            finally:
                r.close()


@pytest.mark.parametrize("env", [{}, {"PT_BOX_PAIRS": "1"}, {"PT_BOX_PAIRS": "1", "PT_PAIR_QUEUE": "16"},
                                 {"PT_BOX_PAIRS": "1", "PT_PAIRS": "0"}])
def test_box_level_pairs_bitexact(ptamd_mod, monkeypatch, env):
    """Box-level pairs in the hipRTC flat kernel (PT_BOX_PAIRS=1, a measured-slower option kept
    for A/B; where every leaf holds one triangle and no distinct leaf box bounds more than two
    leaves): the mask carries one
    bit per distinct box and a (lane, box) pair tests the box's one or two triangles; the
    least (t, rank) wins, in the pair rounds (atomic min) and in the per-lane loops of a queue
    overflow (PT_PAIR_QUEUE=16) or without queues (PT_PAIRS=0). Also a scene whose leaves share
    a box three times (no box-level pairs: leaf pairs as before). Oracle bits and ray counts."""
    import _oracle as O
    from ptamd import scenes
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("PT_RTC_WAIT", "1")
    base = scenes.cornell((36, 30))
    # three triangles with one bounding box (a quad split into three fans) added to Cornell
    fan = [((200.0, 100.0, 300.0), (300.0, 100.0, 300.0), (300.0, 200.0, 300.0)),
           ((200.0, 100.0, 300.0), (300.0, 200.0, 300.0), (200.0, 200.0, 300.0)),
           ((200.0, 100.0, 300.0), (300.0, 100.0, 300.0), (200.0, 200.0, 300.0))]
    triple = scenes.Scene("triple_box", base.camera, list(base.tris) + fan, list(base.mats) + [base.mats[0]] * 3)
    for sc, spp in ((base, 5), (scenes.modified_cornell(0.3, (32, 28)), 4), (triple, 4)):
        img, st = _render(ptamd_mod, sc, spp, 5)
        ref, rays = O.render(sc, spp, 5)
        assert st["kernel_path"] == 3, sc.name
        assert _bits_equal(img, ref) and st["rays"] == rays, (env, sc.name)


def test_devices_reuse_cached_contexts(ptamd_mod, golden_meta):
    """pt_render_*_devices keep their contexts per device list: a second
    render on the same list creates no context; the same scene is not uploaded again, a
    different one is; pt_devices_release frees them and the next call starts fresh. Two
    scenes rendered back to back on the cached contexts give the reference's PNG bytes."""
    names = list(golden_meta["png"])
    names = [next(n for n in names if n.startswith("cornell")), next(n for n in names if n.startswith("mcornell"))]
    ptamd_mod.devices_release()
    jobs = []
    for name in names:  # two different scenes (the camera and resolution are not part of one)
        m = golden_meta["images"][name]
        sc = scene_for(m["scene"], m["res"])
        jobs.append((name, m, ptamd_mod.Camera.from_spec(sc.camera), ptamd_mod.BVH.from_scene(sc)))

    def run(job):
        name, m, cam, bvh = job
        rgb, _ = ptamd_mod.render_rgb8(cam, bvh, m["spp"], m["depth"], devices=[0], band_rows=8)
        assert np.array_equal(rgb, load_golden(name + "_png")), name

    c0, u0, s0 = (ptamd_mod.debug_counter(k) for k in (0, 1, 3))
    run(jobs[0])
    assert ptamd_mod.debug_counter(0) == c0 + 1 and ptamd_mod.debug_counter(1) == u0 + 1
    assert ptamd_mod.debug_counter(2) == 1
    run(jobs[0])  # same list, same scene: no context, no upload
    assert ptamd_mod.debug_counter(0) == c0 + 1 and ptamd_mod.debug_counter(1) == u0 + 1
    assert ptamd_mod.debug_counter(3) == s0 + 1
    run(jobs[1])  # another scene on the cached context: uploaded, no context
    run(jobs[0])
    assert ptamd_mod.debug_counter(0) == c0 + 1 and ptamd_mod.debug_counter(1) == u0 + 3
    m = golden_meta["images"]["cornell_48x40_s8_d8"]  # same scene, another camera: no upload
    sc = scene_for(m["scene"], m["res"])
    rgb, _ = ptamd_mod.render_rgb8(ptamd_mod.Camera.from_spec(sc.camera), ptamd_mod.BVH.from_scene(sc), m["spp"],
                                   m["depth"], devices=[0], band_rows=8)
    assert np.array_equal(rgb, load_golden("cornell_48x40_s8_d8_png"))
    assert ptamd_mod.debug_counter(1) == u0 + 3
    ptamd_mod.devices_release()
    assert ptamd_mod.debug_counter(2) == 0
    run(jobs[1])
    assert ptamd_mod.debug_counter(0) == c0 + 2
    ptamd_mod.devices_release()


@pytest.mark.parametrize("mode", ["1", "2"])
def test_exact_slab_path_bitexact(ptamd_mod, monkeypatch, mode):
    """The kernel's compare-select slab test (taken by waves with a zero direction
    component) gives the same image as the IEEE min/max path. Mode 2 forces it in the
    odd waves of every block only, so exact-walk stacks and the flat path's pair queues
    (which share the LDS stack region) are live in the same block at once."""
    import _oracle as O
    from ptamd import scenes
    sc = scenes.modified_cornell(0.3, (40, 32) if mode == "1" else (96, 80))
    spp = 6 if mode == "1" else 4
    monkeypatch.setenv("PT_FORCE_EXACT_SLAB", mode)
    img, st = _render(ptamd_mod, sc, spp, 5)
    monkeypatch.delenv("PT_FORCE_EXACT_SLAB")
    ref, rays = O.render(sc, spp, 5)
    assert _bits_equal(img, ref) and st["rays"] == rays


def test_pair_queue_matches_per_lane_loop_at_scale(ptamd_mod, monkeypatch):
    """Flat path: the wave-distributed triangle phase (pair queues) and the per-lane
    loop give bit-identical images and ray counts on a specular scene at 1M paths."""
    from ptamd import scenes
    sc = scenes.modified_cornell(0.3, (256, 256))
    img, st = _render(ptamd_mod, sc, 16, 5)
    monkeypatch.setenv("PT_PAIRS", "0")
    img0, st0 = _render(ptamd_mod, sc, 16, 5)
    monkeypatch.delenv("PT_PAIRS")
    assert st["kernel_path"] == st0["kernel_path"] == 3
    assert _bits_equal(img, img0) and st["rays"] == st0["rays"]


def test_narrow_axis_camera_bitexact(ptamd_mod):
    """A near-zero-fov camera looking straight down +z: primary rays are almost
    axis-parallel (tiny x/y direction components, huge inverse directions) and all hit
    the back wall at grazing-free incidence, then bounce around the box."""
    import _oracle as O
    from ptamd import scenes
    base = scenes.cornell((33, 33))
    cam = scenes.CameraSpec((278.0, 274.4, 0.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0), (33, 33), 1e-3, 1.0)
    sc = scenes.Scene("axis", cam, list(base.tris), list(base.mats))
    img, st = _render(ptamd_mod, sc, 3, 5)
    ref, rays = O.render(sc, 3, 5)
    assert _bits_equal(img, ref) and st["rays"] == rays


@pytest.mark.parametrize("env", [{}, {"PT_RTC_DEFINES": "PT_FLAT_SIGN_MASK=1"}, {"PT_RTC": "0"}, {"PT_WIDE": "1"}])
def test_origin_on_box_planes_bitexact(ptamd_mod, monkeypatch, env):
    """Cameras whose position lies ON leaf-box planes of the Cornell box (the floor y = 0,
    the wall x = 0, the opening z = 0), inside the room, with rays leaving through those
    planes: slab values (0 - 0) * (1 / d) = -0 for d < 0, so exit values of -0 reach the box
    test. A sign-bit box mask must treat -0 as 0, as the compare max(tmin, 0) <= tmax does:
    the wide walk's (PT_SIGN_MASK, default) and the hipRTC flat kernel's sign-bit variant
    (tmax + 0; off by default, compiled here with PT_FLAT_SIGN_MASK=1). Bits and
    ray counts against the oracle on the hipRTC flat kernel in both forms, the table flat
    kernel and the wide walk."""
    import _oracle as O
    from ptamd import scenes
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("PT_RTC_WAIT", "1")
    base = scenes.cornell((24, 20))
    for pos, fwd in (((278.0, 0.0, 250.0), (0.1, 0.05, 1.0)), ((0.0, 200.0, 250.0), (0.2, 0.1, 1.0)),
                     ((300.0, 250.0, 0.0), (0.1, -0.2, 1.0))):
        cam = scenes.CameraSpec(pos, fwd, (0.0, 1.0, 0.0), (24, 20), 100.0, 1.0)
        sc = scenes.Scene("plane_cam", cam, list(base.tris), list(base.mats))
        img, st = _render(ptamd_mod, sc, 4, 5)
        ref, rays = O.render(sc, 4, 5)
        assert st["kernel_path"] == (4 if env.get("PT_WIDE") else 5 if env.get("PT_RTC") else 3)
        assert _bits_equal(img, ref) and st["rays"] == rays, (pos, env)


def test_deterministic_and_edge_params(ptamd_mod):
    from ptamd import scenes
    sc = scenes.cornell((16, 16))
    a, _ = _render(ptamd_mod, sc, 5, 5)
    b, _ = _render(ptamd_mod, sc, 5, 5)
    assert _bits_equal(a, b)
    z, st = _render(ptamd_mod, sc, 4, 0)  # depth 0: trace() returns 0, no rays
    assert st["rays"] == 0 and np.all(z == 0)
    n, st = _render(ptamd_mod, sc, 0, 5)  # spp 0: 0 / 0 (render.h:97)
    assert np.all(np.isnan(n)) and st["rays"] == 0
    c, _ = _render(ptamd_mod, sc, 3, 5, seed=7)
    import _oracle as O
    ref, _ = O.render(sc, 3, 5, seed=7)
    assert _bits_equal(c, ref)


def test_device_math_matches_oracle(ptamd_mod):
    import ctypes as C
    import _oracle as O
    rng = np.random.default_rng(5)
    lib = ptamd_mod.lib()
    # acosf over (2u-1) for u = rand01 values, plus edges
    st = rng.integers(0, 2**32, size=1 << 20, dtype=np.uint64).astype(np.uint32)
    u = (st.astype(np.float32) * np.float32(2.0 ** -32)).astype(np.float32)
    x = np.concatenate([(np.float32(2) * u - np.float32(1)).astype(np.float32),
                        np.array([-1, 1, 0, -0.0, 0.5, -0.5, 1e-9, -1e-9, 2, np.nan], np.float32),
                        rng.uniform(-1, 1, 1 << 20).astype(np.float32)])
    x = np.ascontiguousarray(x)
    gpu = np.empty_like(x)
    assert lib.pt_debug_math(0, 0, x.ctypes.data, x.size, gpu.ctypes.data) == 0
    ref = np.empty_like(x)
    O.lib().oracle_acosf_n(x.ctypes.data_as(C.c_void_p), x.size, ref.ctypes.data_as(C.c_void_p))
    assert _bits_equal(gpu, ref)
    # sincosf over theta in [-pi/2, pi/2] and phi in [0, 2pi]
    y = np.ascontiguousarray(np.concatenate([rng.uniform(-1.6, 1.6, 1 << 20), rng.uniform(0, 6.3, 1 << 20),
                                             [0.0, -0.0, 1e-5, 0.785, 0.7854, 3.1415927, 6.2831855]]).astype(np.float32))
    g2 = np.empty(2 * y.size, np.float32)
    assert lib.pt_debug_math(0, 1, y.ctypes.data, y.size, g2.ctypes.data) == 0
    s = np.empty_like(y)
    c = np.empty_like(y)
    O.lib().oracle_sincosf_n(y.ctypes.data_as(C.c_void_p), y.size, s.ctypes.data_as(C.c_void_p),
                             c.ctypes.data_as(C.c_void_p))
    assert _bits_equal(g2[0::2], s) and _bits_equal(g2[1::2], c)


def test_device_brdf_matches_oracle(ptamd_mod):
    import ctypes as C
    import _oracle as O
    rng = np.random.default_rng(9)
    n = 4096
    items = np.zeros((n, 9), np.float32)
    states = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    types = np.where(np.arange(n) % 2 == 0, 2, 3).astype(np.int32)
    rough = rng.choice([0.0, 0.05, 0.3, 0.8, 2.0], size=n).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    nn = rng.normal(size=(n, 3)).astype(np.float32)
    nn /= np.linalg.norm(nn, axis=1, keepdims=True)
    flip = (d * nn).sum(1) >= 0
    nn[flip] *= -1  # face-forward, as trace() passes it
    items[:, 0] = states.view(np.float32)
    items[:, 1] = types.view(np.float32)
    items[:, 2] = rough
    items[:, 3:6] = d
    items[:, 6:9] = nn
    items = np.ascontiguousarray(items)
    out = np.empty((n, 4), np.float32)
    assert ptamd_mod.lib().pt_debug_math(0, 2, items.ctypes.data, n, out.ctypes.data) == 0
    for i in range(n):
        r = np.empty(3, np.float32)
        st = O.lib().oracle_brdf(int(states[i]), int(types[i]), C.c_float(rough[i]),
                                 np.ascontiguousarray(d[i]).ctypes.data_as(C.c_void_p),
                                 np.ascontiguousarray(nn[i]).ctypes.data_as(C.c_void_p), r.ctypes.data_as(C.c_void_p))
        assert _bits_equal(out[i, :3], r), i
        assert out[i, 3:4].view(np.uint32)[0] == st, i


@pytest.mark.parametrize("which", [0, 1])
def test_fast_exact_math_sweep(ptamd_mod, which):
    """rcp_exact / sqrt_exact (pt_math.h) equal the IEEE 1/x and sqrt(x) on EVERY float:
    the fast sequences on their proven ranges, the guarded IEEE fallback elsewhere.
    (All 2^32 bit patterns, NaNs skipped; ~0.1 s on the GPU.)"""
    import ctypes as C
    lib = ptamd_mod.lib()
    bad, first = C.c_uint64(0), C.c_uint32(0)
    assert lib.pt_debug_sweep(0, which, 0, 0xFFFFFFFF, C.byref(bad), C.byref(first)) == 0, lib.pt_last_error()
    assert bad.value == 0, f"{bad.value} mismatches, first input bits 0x{first.value:08x}"
    assert first.value == 0xFFFFFFFF


def test_fast_division_sweep(ptamd_mod):
    """div_by_rcp (Markstein's correction on the correctly rounded reciprocal, used by the
    camera's normalize) equals IEEE x / b for every float x with |x| in [2^-60, 2^60],
    each against a hashed divisor from the camera-length range [1, 2^11) or from
    [2^-60, 2^60] (2^32 inputs, ~2^31 of them in range)."""
    import ctypes as C
    lib = ptamd_mod.lib()
    bad, first = C.c_uint64(0), C.c_uint32(0)
    assert lib.pt_debug_sweep(0, 4, 0, 0xFFFFFFFF, C.byref(bad), C.byref(first)) == 0, lib.pt_last_error()
    assert bad.value == 0, f"{bad.value} mismatches, first input bits 0x{first.value:08x}"


@pytest.mark.parametrize("which,lo,hi", [(2, 0x00000000, 0x3F800000), (2, 0x80000000, 0xBF800000),
                                         (3, 0x00000000, 0x40E00000), (3, 0x80000000, 0xC0000000)])
def test_fast_libm_sweep(ptamd_mod, which, lo, hi):
    """The device's fast acosf (Markstein-corrected division, rcp_exact, sqrt_exact) and
    sincosf (FMA-contracted double kernel) equal the glibc restatements on every float of
    the path's domain: acosf on [-1, 1] (argument 2u - 1), sincosf on [-2, 7] (theta in
    [-pi/2, pi/2], phi in [0, 2pi]), so the hemisphere sample stays bit-exact."""
    import ctypes as C
    lib = ptamd_mod.lib()
    bad, first = C.c_uint64(0), C.c_uint32(0)
    assert lib.pt_debug_sweep(0, which, lo, hi, C.byref(bad), C.byref(first)) == 0, lib.pt_last_error()
    assert bad.value == 0, f"{bad.value} mismatches, first input bits 0x{first.value:08x}"


def test_pair_queue_overflow_fallback_bitexact(ptamd_mod, monkeypatch):
    """A wave whose (lane, leaf) pairs exceed its queue takes the per-lane loop for that
    iteration (rare at the default 512 entries per wave; forced here with 16)."""
    import _oracle as O
    from ptamd import scenes
    monkeypatch.setenv("PT_PAIR_QUEUE", "16")
    for sc, spp, depth in [(scenes.cornell((40, 33)), 5, 5), (scenes.modified_cornell(0.3, (32, 32)), 4, 5)]:
        img, st = _render(ptamd_mod, sc, spp, depth)
        ref, rays = O.render(sc, spp, depth)
        assert _bits_equal(img, ref) and st["rays"] == rays, sc.name


@pytest.mark.parametrize("thresh", ["1", "64"])
def test_camera_prefetch_threshold_invariance(ptamd_mod, monkeypatch, thresh):
    """Camera rays generated one path ahead: any refill threshold gives the same bits."""
    import _oracle as O
    from ptamd import scenes
    monkeypatch.setenv("PT_REGEN_THRESH", thresh)
    sc = scenes.cornell((48, 45))
    img, st = _render(ptamd_mod, sc, 12, 5)
    ref, rays = O.render(sc, 12, 5)
    assert _bits_equal(img, ref) and st["rays"] == rays


# ------------------------------------------------------- §8(f): device post-process, progressive
@pytest.mark.parametrize("gamma", [2.2, 1.0, 0.5, 3.0])
def test_device_quantiser_matches_oracle(ptamd_mod, gamma):
    """pt_rgb8_kernel (LDS threshold search) == gamma_correct + save_png bytes (oracle,
    pinned to the reference's PNGs by test_rgb8.py) on every threshold +-4 ulps, the
    special values and a random spread, in a ragged 1-row and a 2-D layout."""
    import _oracle as O
    from test_rgb8 import _neighbourhood
    thr, _ = ptamd_mod.rgb8_thresholds(gamma)
    x = _neighbourhood(thr)
    n = -(-x.size // 3)
    flat = np.zeros(3 * n, np.float32)
    flat[: x.size] = x
    for shape in ((1, n, 3), (n // 37, 37, 3)):
        img = flat[: int(np.prod(shape))].reshape(shape)
        assert np.array_equal(ptamd_mod.device_rgb8(img, gamma), O.rgb8(img, gamma)), shape


def test_render_rgb8_matches_reference_png(ptamd_mod, golden_meta):
    """pt_ctx_render_rgb8 == the reference's own PNG bytes (render.h:97-100)."""
    for name in golden_meta["png"]:
        m = golden_meta["images"][name]
        sc = scene_for(m["scene"], m["res"])
        r = ptamd_mod.Renderer(0)
        r.set_scene(ptamd_mod.BVH.from_scene(sc))
        rgb, st = r.render_rgb8(ptamd_mod.Camera.from_spec(sc.camera), m["spp"], m["depth"])
        r.close()
        assert np.array_equal(rgb, load_golden(name + "_png")), name
        assert st["paths"] == m["res"][0] * m["res"][1] * m["spp"]


def test_render_rgb8_parts_and_device_output(ptamd_mod):
    """Row partition + flip=0 keeps pt_ctx_render's row order; a torch uint8 device
    tensor receives the same bytes."""
    import torch
    import _oracle as O
    sc = scene_for("cornell", [40, 24])
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    r = ptamd_mod.Renderer(0)
    r.set_scene(ptamd_mod.BVH.from_scene(sc))
    for part in range(3):
        lin, _ = r.render(cam, 4, 5, part_index=part, part_count=3, band_rows=4)
        rgb, _ = r.render_rgb8(cam, 4, 5, flip=False, part_index=part, part_count=3, band_rows=4)
        assert np.array_equal(rgb, O.rgb8(lin)[::-1]), part
        dev = torch.empty(rgb.size, dtype=torch.uint8, device="cuda:0")
        r.render_rgb8(cam, 4, 5, flip=False, part_index=part, part_count=3, band_rows=4, out=dev)
        assert np.array_equal(dev.cpu().numpy().reshape(rgb.shape), rgb), part
    r.close()


def test_progressive_frames_equal_one_shot_renders(ptamd_mod, golden_meta):
    """Frame accumulation: after each frame the running mean equals a one-shot render of
    that many samples (per-sample seeds + in-order sums), ending on the golden image;
    a frame that does not continue the sum is refused."""
    m = golden_meta["images"]["cornell_64_s16_d5"]
    sc = scene_for(m["scene"], m["res"])
    bvh = ptamd_mod.BVH.from_scene(sc)
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    prog, one = ptamd_mod.Renderer(0), ptamd_mod.Renderer(0)
    prog.set_scene(bvh)
    one.set_scene(bvh)
    s = 0
    for k in (1, 2, 0, 5, 8):
        img, st = prog.render_progressive(cam, s, k, 5, batch_spp=3)
        s += k
        want, _ = one.render(cam, s, 5)
        assert _bits_equal(img, want), s
        assert st["paths"] == k * 64 * 64
    assert s == 16 and _bits_equal(img, load_golden("cornell_64_s16_d5"))
    with pytest.raises(ptamd_mod.PTError):
        prog.render_progressive(cam, 5, 1, 5)  # not the running sum's length
    with pytest.raises(ptamd_mod.PTError):
        prog.render_progressive(cam, 16, 1, 3)  # another depth
    img, _ = prog.render_progressive(cam, 16, 4, 5)  # a refused call leaves the sum intact
    want, _ = one.render(cam, 20, 5)
    assert _bits_equal(img, want)
    prog.render(cam, 2, 5)  # any other render ends the sum
    with pytest.raises(ptamd_mod.PTError):
        prog.render_progressive(cam, 20, 1, 5)
    prog.close()
    one.close()


def test_obj_mesh_render_bitexact(ptamd_mod, golden_meta):
    """An OBJ scene (quads + polygon caps) loaded by BVH.load_obj renders bit-identical
    to the reference's load_obj + render of the same file (tests/golden/gen_obj.py)."""
    import os
    from ptamd import scenes
    m = golden_meta["obj"]["files"]["mesh"]["render"]
    obj_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "obj")
    bvh = ptamd_mod.BVH()
    bvh.load_obj(os.path.join(obj_dir, "mesh.obj"), obj_dir)
    cam = ptamd_mod.Camera.from_spec(scenes.CameraSpec((278.0, 278.0, -500.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0),
                                                       tuple(m["res"]), 60.0, 1.0))
    img, st = ptamd_mod.render(cam, bvh, m["spp"], m["depth"])
    assert _bits_equal(img, load_golden("obj_mesh_img"))
    assert st["paths"] == m["res"][0] * m["res"][1] * m["spp"]


@pytest.mark.parametrize("case", ["exact1", "exact2", "smallq"])
def test_wide_walk_exact_and_queue_fallbacks(ptamd_mod, monkeypatch, case):
    """Wide path: the exact binary walk (stacks in HBM) for forced waves, and a tiny
    triangle queue (PT_WIDE_QUEUE_CAP=8: early drains and the per-lane fallback when a
    step's leaves exceed it) give the oracle's bits and ray count."""
    import _oracle as O
    from ptamd import scenes
    monkeypatch.setenv("PT_WIDE", "1")
    if case.startswith("exact"):
        monkeypatch.setenv("PT_FORCE_EXACT_SLAB", case[-1])
    else:
        monkeypatch.setenv("PT_WIDE_QUEUE_CAP", "8")
    for sc, spp in ((scenes.sphere_in_cornell(32, (48, 40)), 3), (scenes.modified_cornell(0.3, (40, 32)), 4)):
        img, st = _render(ptamd_mod, sc, spp, 5)
        ref, rays = O.render(sc, spp, 5)
        assert st["kernel_path"] == 4, sc.name
        assert _bits_equal(img, ref) and st["rays"] == rays, (case, sc.name)


@pytest.mark.parametrize("devices,gather", [([0], "none"), ([0], "rccl"), ([0, 0, 0], "host"), ([0], "host")])
def test_multi_device_one_shot_bitexact(ptamd_mod, golden_meta, monkeypatch, devices, gather):
    """pt_render_f32_devices: row bands rendered by one context (and host thread) per
    listed device, bit-identical to the reference. One device: its part is the frame (no
    gather, RCCL never loaded). Distinct devices meet through the RCCL leg —
    ncclCommInitAll, one ncclSend/ncclRecv group to device 0, rows assembled on the device
    (forced on the box's one GPU with PT_GATHER=rccl: RCCL's send-to-self); a device listed
    3 times, or PT_GATHER=host, through host assembly. Per-device stats add up."""
    if len(devices) == 1 and gather != "none":
        monkeypatch.setenv("PT_GATHER", gather)
    for name in ("cornell_48x40_s8_d8", "mcornell_r0.3_64_s8_d5"):
        m = golden_meta["images"][name]
        sc = scene_for(m["scene"], m["res"])
        img, st = ptamd_mod.render(ptamd_mod.Camera.from_spec(sc.camera), ptamd_mod.BVH.from_scene(sc), m["spp"],
                                   m["depth"], devices=devices, band_rows=4)
        assert _bits_equal(img, load_golden(name)), (name, devices)
        assert st["paths"] == m["res"][0] * m["res"][1] * m["spp"]
        assert ptamd_mod._lib.pt_stats.GATHERS[st["gather_path"]] == gather
        assert st["n_devices"] == len(devices) and sum(st["device_rays"]) == st["rays"]
        assert max(st["device_kernel_ms"]) == st["kernel_ms"]


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_multi_device_rgb8_matches_reference_png(ptamd_mod, golden_meta, devices):
    """pt_render_rgb8_devices: gather, then gamma + quantisation on the first device —
    the reference's own PNG bytes (render.h:97-100, image.h:41-62)."""
    for name in golden_meta["png"]:
        m = golden_meta["images"][name]
        sc = scene_for(m["scene"], m["res"])
        rgb, st = ptamd_mod.render_rgb8(ptamd_mod.Camera.from_spec(sc.camera), ptamd_mod.BVH.from_scene(sc),
                                        m["spp"], m["depth"], devices=devices, band_rows=8)
        assert np.array_equal(rgb, load_golden(name + "_png")), (name, devices)


def test_hooks_ignored_without_gate(ptamd_mod, tmp_path):
    """Test hooks are read only under PT_TEST_HOOKS=1: in a process without the gate,
    PT_FLAT=0 / PT_PAIRS=0 do not change the kernel (a flat-path kernel still runs: the
    generic one while the hipRTC kernel compiles in the background, or the hipRTC one)."""
    import json
    import os
    import subprocess
    import sys
    code = ("import sys, json; sys.path.insert(0, %r); import ptamd; from ptamd import scenes; "
            "sc = scenes.cornell((16, 16)); img, st = ptamd.render(ptamd.Camera.from_spec(sc.camera), "
            "ptamd.BVH.from_scene(sc), 2, 5); print(json.dumps(st['kernel_path']))"
            % os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pathtracer-cpp_amd"))
    env = {k: v for k, v in os.environ.items() if k != "PT_TEST_HOOKS"}
    env.update(PT_FLAT="0", PT_PAIRS="0")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert json.loads(out.stdout.strip().splitlines()[-1]) in (3, 5)  # PT_PATH_FLAT_RTC / _TABLE_FAST


@pytest.mark.parametrize("sync", ["0", "1"])
def test_context_stream_made_on_a_thread(ptamd_mod, monkeypatch, sync):
    """pt_ctx_create makes the context's stream and work counter on a thread of its own
    (round 6: ~5 ms that overlap the scene packing); every entry point joins it first. Contexts
    destroyed at once, prepared without a scene, or rendered right after creation work as with
    the stream made in pt_ctx_create (PT_CTX_SYNC=1), with the oracle's bits."""
    import _oracle as O
    from ptamd import scenes
    monkeypatch.setenv("PT_CTX_SYNC", sync)
    for _ in range(8):  # destroyed while its init thread may still run
        ptamd_mod.Renderer(0).close()
    r = ptamd_mod.Renderer(0)
    try:
        r.prepare()  # no scene: nothing to wait for but the stream
    finally:
        r.close()
    sc = scenes.cornell((16, 16))
    img, st = _render(ptamd_mod, sc, 2, 4)
    ref, rays = O.render(sc, 2, 4)
    assert _bits_equal(img, ref) and st["rays"] == rays
    sc4 = scenes.sphere_in_cornell(24, (16, 16))  # a wide-tree scene (its packing runs on threads)
    monkeypatch.setenv("PT_WIDE", "1")
    img4, st4 = _render(ptamd_mod, sc4, 2, 3)
    ref4, rays4 = O.render(sc4, 2, 3)
    assert _bits_equal(img4, ref4) and st4["rays"] == rays4


def test_rtc_background_compile(ptamd_mod, monkeypatch):
    """Library default: pt_ctx_set_scene starts the hipRTC compile in the background. A
    render right after it runs the generic flat kernel while the compile is still going and
    switches to the hipRTC kernel between launches once it is done; both kernels give the
    same bits."""
    import _oracle as O
    from ptamd import scenes
    monkeypatch.setenv("PT_RTC_WAIT", "0")
    sc = scenes.cornell((32, 32))
    a, b, c = sc.tris[0]
    sc.tris[0] = ((a[0] + 0.25, a[1], a[2]), b, c)  # a scene (so a hipRTC source) no other test compiles
    bvh = ptamd_mod.BVH.from_scene(sc)
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    r = ptamd_mod.Renderer(0)
    try:
        r.set_scene(bvh)
        img0, st0 = r.render(cam, 4, 5)
        assert st0["kernel_path"] in (3, 5)
        ref, rays = O.render(sc, 4, 5)
        assert _bits_equal(img0, ref) and st0["rays"] == rays
        big = ptamd_mod.Camera.from_spec(sc.with_res(1024, 1024).camera)
        _, st1 = r.render(big, 256, 2)  # switches to the hipRTC kernel between launches once compiled
        assert st1["kernel_path"] in (3, 5)
        r.prepare()  # waits for the compile
        img2, st2 = r.render(cam, 4, 5)
        assert st2["kernel_path"] == 3 and _bits_equal(img2, img0) and st2["rays"] == st0["rays"]
    finally:
        r.close()


def test_rtc_disk_cache_first_launch_and_corrupt_entry(ptamd_mod, monkeypatch, tmp_path):
    """The on-disk code-object cache: once a scene's kernel is compiled, a process that
    meets the scene again (here: after forgetting its own compiles) starts its FIRST launch
    on the hipRTC kernel (no background compile, no generic-kernel launches), and a
    corrupted entry is rejected and recompiled; the bits are the oracle's throughout."""
    import _oracle as O
    from ptamd import scenes
    monkeypatch.setenv("PT_RTC_WAIT", "0")
    monkeypatch.setenv("PT_RTC_CACHE_DIR", str(tmp_path))
    L = ptamd_mod.lib()
    sc = scenes.cornell((40, 30))
    a, b, c = sc.tris[2]
    sc.tris[2] = ((a[0] - 0.125, a[1], a[2]), b, c)  # a hipRTC source no other test compiles
    bvh = ptamd_mod.BVH.from_scene(sc)
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    ref, rays = O.render(sc, 5, 5)

    def fresh_render():
        L.pt_debug_rtc_cache(0)
        r = ptamd_mod.Renderer(0)
        try:
            r.set_scene(bvh)
            img, st = r.render(cam, 5, 5)
            r.prepare()
            img2, st2 = r.render(cam, 5, 5)
        finally:
            r.close()
        assert _bits_equal(img, ref) and st["rays"] == rays
        assert _bits_equal(img2, ref) and st2["kernel_path"] == 3
        return st

    c0 = L.pt_debug_rtc_cache(3)
    fresh_render()  # compiles (background), stores the entry
    entries = list(tmp_path.glob("*.co"))
    assert L.pt_debug_rtc_cache(3) == c0 + 1 and len(entries) == 1
    h0 = L.pt_debug_rtc_cache(1)
    st = fresh_render()  # the verified entry: the first launch is already the hipRTC kernel
    assert st["kernel_path"] == 3 and L.pt_debug_rtc_cache(1) == h0 + 1 and L.pt_debug_rtc_cache(3) == c0 + 1
    data = bytearray(entries[0].read_bytes())
    data[len(data) // 2] ^= 0x5A
    entries[0].write_bytes(bytes(data))
    r0 = L.pt_debug_rtc_cache(2)
    fresh_render()  # rejected, recompiled, rewritten; the generic kernel meanwhile
    assert L.pt_debug_rtc_cache(2) == r0 + 1 and L.pt_debug_rtc_cache(3) == c0 + 2
    st = fresh_render()
    assert st["kernel_path"] == 3 and L.pt_debug_rtc_cache(1) == h0 + 2


@pytest.mark.parametrize("at", [1, 3])
def test_rtc_switch_within_a_frame_bitexact(ptamd_mod, monkeypatch, at):
    """A frame whose first launches run the generic flat kernel and the rest the hipRTC
    kernel (the switch forced at launch `at`, PT_RTC_SWITCH_AT; small batches, so the frame
    has several launches with fused accumulation) gives the oracle's bits and ray count."""
    import _oracle as O
    from ptamd import scenes
    monkeypatch.setenv("PT_RTC_WAIT", "0")
    monkeypatch.setenv("PT_RTC_SWITCH_AT", str(at))
    sc = scenes.modified_cornell(0.3, (24, 20))
    a, b, c = sc.tris[1]
    sc.tris[1] = ((a[0] + 0.125 * at, a[1], a[2]), b, c)  # a hipRTC source no other test compiles
    bvh = ptamd_mod.BVH.from_scene(sc)
    cam = ptamd_mod.Camera.from_spec(sc.camera)
    r = ptamd_mod.Renderer(0)
    try:
        r.set_scene(bvh)
        img, st = r.render(cam, 10, 5, batch_spp=2)
        assert st["kernel_path"] == 3 and st["trace_launches"] == 5
        ref, rays = O.render(sc, 10, 5)
        assert _bits_equal(img, ref) and st["rays"] == rays
    finally:
        r.close()


def test_multi_device_concurrent_calls_share_communicators(ptamd_mod, golden_meta, monkeypatch):
    """Two host threads render over the same device list at once through the RCCL leg
    (PT_GATHER=rccl on the box's one GPU): the cached communicators are locked per group
    (pt_multi.hip, CommSet::mu), so both frames come out bit-exact."""
    import threading
    monkeypatch.setenv("PT_GATHER", "rccl")
    m = golden_meta["images"]["cornell_48x40_s8_d8"]
    sc = scene_for(m["scene"], m["res"])
    out, errs = {}, []

    def run(i):
        try:
            out[i] = ptamd_mod.render(ptamd_mod.Camera.from_spec(sc.camera), ptamd_mod.BVH.from_scene(sc), m["spp"],
                                      m["depth"], devices=[0], band_rows=4)
        except Exception as e:  # noqa: BLE001 — reported below
            errs.append(e)

    for _ in range(3):
        th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not errs and len(out) == 2
        for img, st in out.values():
            assert _bits_equal(img, load_golden("cornell_48x40_s8_d8"))
            assert ptamd_mod._lib.pt_stats.GATHERS[st["gather_path"]] == "rccl"
        out.clear()


@pytest.mark.parametrize("seed,n_tris", [(1, 20), (2, 40), (3, 50), (4, 150), (5, 300)])
def test_random_scenes_bitexact(ptamd_mod, monkeypatch, seed, n_tris):
    """Seeded random scenes (random triangles, materials and camera inside a closed room) on
    every kernel path that takes them: the hipRTC scene kernel and the generic flat kernel
    (<= 64 leaves), the wide walk and the binary-tree walk: the oracle's bits and ray counts."""
    import _oracle as O
    from _randscene import random_scene
    sc = random_scene(seed, n_tris, (26, 21))
    ref, rays = O.render(sc, 3, 5)
    flat = n_tris + 12 <= 64
    envs = ([{"PT_RTC_WAIT": "1"}, {"PT_RTC": "0"}] if flat else [{}]) + [{"PT_FLAT": "0"}, {"PT_FLAT": "0", "PT_WIDE": "0"}]
    for env in envs:
        with monkeypatch.context() as m:
            for k, v in env.items():
                m.setenv(k, v)
            img, st = _render(ptamd_mod, sc, 3, 5)
            assert _bits_equal_nan(img, ref) and st["rays"] == rays, (seed, env)
