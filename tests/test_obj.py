"""OBJ/MTL ingestion (BVH::load_obj, bvh.h:184-242).

The product reader (csrc/pt_obj.cpp behind pt_obj_load, used by ptamd.BVH.load_obj
and the drop-in header) against what the reference itself loaded from the same
files (tests/golden/gen_obj.py: oracle/_ref/pt_ref --obj, i.e. the reference's
vendored tinyobjloader): triangle vertices and Material bytes bit-exact, in order,
and the reference's BVH::build of them. Bar: bit-exact.
"""
import os

import numpy as np
import pytest

from conftest import load_golden

OBJ_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "obj")
NAMES = ["edge", "numbers", "polys", "mesh"]


def _load(name):
    import ptamd
    b = ptamd.BVH()
    b.load_obj(os.path.join(OBJ_DIR, name + ".obj"), OBJ_DIR)
    return b


@pytest.mark.parametrize("name", NAMES)
def test_triangles_match_reference(golden_meta, name, capfd):
    b = _load(name)
    err = capfd.readouterr().err
    ref_v = load_golden(f"obj_{name}_verts")
    ref_m = load_golden(f"obj_{name}_mats")
    assert b.size() == ref_v.shape[0] == golden_meta["obj"]["files"][name]["tris"]
    assert b.verts().tobytes() == ref_v.tobytes()
    assert bytes(b.materials()) == ref_m.tobytes()
    assert err.count("Unknown material type with illum") == golden_meta["obj"]["files"][name]["unknown_material_msgs"]


@pytest.mark.parametrize("name", NAMES)
def test_bvh_of_obj_matches_reference(name):
    b = _load(name)
    b.build()
    assert b.nodes.tobytes() == load_golden(f"obj_{name}_nodes").tobytes()
    assert np.array_equal(b.tri_idx, load_golden(f"obj_{name}_idx"))


def test_edge_cases_are_covered():
    """The edge fixture reaches the reader's branches: quads split both ways, ear
    clipping, a map_Kd default, first-definition-wins, CRLF lines, relative indices."""
    import ptamd
    b = _load("edge")
    cols = {tuple(t.material.color) for t in b.triangles}
    emits = {tuple(t.material.emit_color) for t in b.triangles}
    assert (0.75, 0.5, 0.25) in cols            # "white" from edge.mtl, not lib2.mtl's blue
    assert (0.0, 0.0, 1.0) not in cols
    assert tuple(np.float32([0.6] * 3).tolist()) in cols  # map_Kd without Kd in its file
    assert (0.5, 0.5, 0.5) in cols              # illum 3 / missing illum -> Diffuse(0.5)
    assert (4.0, 3.5, 2.0) in emits and (1.0, 1.0, 1.0) in emits
    assert {t.material.type for t in b.triangles} == {ptamd.Material.DIFFUSE, ptamd.Material.EMIT}


@pytest.mark.parametrize("name,msg", [("nomtl", "no material"), ("badidx", "beyond"),
                                      ("zeroidx", "Failed to parse")])
def test_undefined_or_failing_inputs_raise(name, msg):
    import ptamd
    with pytest.raises(ptamd.PTError, match=msg):
        _load(name)


def test_missing_file_raises():
    import ptamd
    with pytest.raises(ptamd.PTError, match="Cannot open file"):
        ptamd.BVH().load_obj(os.path.join(OBJ_DIR, "no_such.obj"))


def test_oracle_render_of_obj_mesh_matches_reference(golden_meta):
    """The CPU oracle on the loaded triangles reproduces the reference's render of
    mesh.obj (the GPU test compares the HIP path with the same fixture)."""
    import _oracle as O
    from ptamd import scenes
    m = golden_meta["obj"]["files"]["mesh"]["render"]
    b = _load("mesh")
    sc = scenes.Scene("obj_mesh", scenes.CameraSpec((278.0, 278.0, -500.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0),
                                                    tuple(m["res"]), 60.0, 1.0))
    for t in b.triangles:
        mt = t.material
        sc.add([(t.v1, t.v2, t.v3)], scenes.Material(mt.type, tuple(mt.color), tuple(mt.emit_color), mt.roughness))
    img, _ = O.render(sc, m["spp"], m["depth"])
    assert img.view(np.uint32).tobytes() == load_golden("obj_mesh_img").view(np.uint32).tobytes()
