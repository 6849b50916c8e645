"""Workload scenes.

The scenes are data: triangle vertices, materials and camera placement of the
reference's example programs, kept here in our own table form.

* ``cornell()``            examples/cornell_box.cc:11-98      (32 tris, configs 1, 2, 5)
* ``modified_cornell(r)``  examples/modified_cornell.cc:12-106 (34 tris, config 3)
* ``tri3()``               tests/test_render.cc:11-21          (3 tris)
* ``sphere_in_cornell(st)`` synthetic UV sphere inside C (config 4, no counterpart
  in the reference; SURVEY.md §8(d) "S")

Vertex order inside each triangle matters (Möller–Trumbore edges and the
normal are taken from v1, triangle.h:28-29, 46), so quads are split exactly as
the examples split them: ``_split_a`` = (p1,p2,p3),(p4,p3,p1) and
``_split_b`` = (p1,p2,p3),(p1,p3,p4).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

EMIT, DIFFUSE, SPECULAR = 1, 2, 3  # Material::Type, material.h:28-32

Vec = Tuple[float, float, float]


@dataclass(frozen=True)
class Material:
    type: int
    color: Vec
    emit: Vec
    roughness: float = 0.0

    @staticmethod
    def make(type_: int, color, emit, roughness=0.0) -> "Material":
        def v(x):
            return (float(x),) * 3 if isinstance(x, (int, float)) else tuple(float(c) for c in x)
        return Material(type_, v(color), v(emit), float(roughness))


@dataclass(frozen=True)
class CameraSpec:
    pos: Vec
    forward: Vec
    up: Vec
    res: Tuple[int, int]
    fov_deg: float
    distance: float = 1.0

    @property
    def fov(self) -> float:
        """Radians, computed as ``deg * DEG2RAD`` = ``(deg * M_PI) / 180`` (linalg.h:10)."""
        return self.fov_deg * math.pi / 180


@dataclass
class Scene:
    name: str
    camera: CameraSpec
    tris: List[Tuple[Vec, Vec, Vec]] = field(default_factory=list)
    mats: List[Material] = field(default_factory=list)

    def add(self, tris: Sequence[Tuple[Vec, Vec, Vec]], mat: Material) -> None:
        for t in tris:
            self.tris.append(t)
            self.mats.append(mat)

    def with_res(self, w: int, h: int) -> "Scene":
        cam = CameraSpec(self.camera.pos, self.camera.forward, self.camera.up, (w, h),
                         self.camera.fov_deg, self.camera.distance)
        return Scene(self.name, cam, list(self.tris), list(self.mats))

    def to_ptscene(self) -> str:
        """Text form read by the reference harness (oracle/ref/pt_ref_harness.cc)."""
        c = self.camera
        r = repr
        lines = [f"# {self.name}",
                 "camera " + " ".join(r(float(x)) for x in (*c.pos, *c.forward, *c.up))
                 + f" {c.res[0]} {c.res[1]} {r(float(c.fov_deg))} {r(float(c.distance))}"]
        for (a, b, cc), m in zip(self.tris, self.mats):
            lines.append("tri " + " ".join(r(float(x)) for x in (*a, *b, *cc))
                         + f" {m.type} " + " ".join(r(float(x)) for x in (*m.color, *m.emit))
                         + f" {r(float(m.roughness))}")
        return "\n".join(lines) + "\n"


def _split_a(p1, p2, p3, p4):
    return [(p1, p2, p3), (p4, p3, p1)]


def _split_b(p1, p2, p3, p4):
    return [(p1, p2, p3), (p1, p3, p4)]


# Room shell of the Cornell scenes (corner points of each wall quad).
_FLOOR = ((552.8, 0, 0), (0, 0, 0), (0, 0, 559.2), (549.6, 0, 559.2))
_LIGHT = ((343, 548.7, 227), (343, 548.7, 332), (213, 548.7, 332), (213, 548.7, 227))
_CEIL = ((556, 548.8, 0), (0, 548.8, 0), (0, 548.8, 559.2), (556.0, 548.8, 559.2))
_BACK = ((549.6, 0, 559.2), (0, 0, 559.2), (0, 548.8, 559.2), (556, 548.8, 559.2))
_FRONT = ((556, 0, 0), (0, 0, 0), (0, 548.8, 0), (556, 548.8, 0))
_RIGHT = ((0, 0, 559.2), (0, 0, 0), (0, 548.8, 0), (0, 548.8, 559.2))
_LEFT = ((552.8, 0, 0), (549.6, 0, 559.2), (556, 548.8, 559.2), (556, 548.8, 0))
_SHORT_BOX = (
    ((130, 165, 65), (82, 165, 225), (240, 165, 272), (290, 165, 114)),
    ((290, 0, 114), (290, 165, 114), (240, 165, 272), (240, 0, 272)),
    ((130, 0, 65), (130, 165, 65), (290, 165, 114), (290, 0, 114)),
    ((82, 0, 225), (82, 165, 225), (130, 165, 65), (130, 0, 65)),
    ((240, 0, 272), (240, 165, 272), (82, 165, 225), (82, 0, 225)),
)
_TALL_BOX = (
    ((423, 330, 247), (265, 330, 296), (314, 330, 456), (472, 330, 406)),
    ((423, 0, 247), (423, 330, 247), (472, 330, 406), (472, 0, 406)),
    ((472, 0, 406), (472, 330, 406), (314, 330, 456), (314, 0, 456)),
    ((314, 0, 456), (314, 330, 456), (265, 330, 296), (265, 0, 296)),
    ((265, 0, 296), (265, 330, 296), (423, 330, 247), (423, 0, 247)),
)


def _fl(q):
    return tuple(tuple(float(c) for c in p) for p in q)


def cornell(res: Tuple[int, int] = (1024, 1024)) -> Scene:
    """examples/cornell_box.cc: 32 triangles, camera at (278,278,-500)."""
    white = Material.make(DIFFUSE, 1, 0, 0)
    light = Material.make(EMIT, 0, 1, 0)
    green = Material.make(DIFFUSE, (0, 1, 0), 0, 0)
    red = Material.make(DIFFUSE, (1, 0, 0), 0, 0)
    s = Scene("cornell", CameraSpec((278.0, 278.0, -500.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0),
                                    tuple(res), 60.0, 1.0))
    s.add(_split_a(*_fl(_FLOOR)), white)
    s.add(_split_a(*_fl(_LIGHT)), light)
    s.add(_split_a(*_fl(_CEIL)), white)
    s.add(_split_a(*_fl(_BACK)), white)
    s.add(_split_a(*_fl(_RIGHT)), green)
    s.add(_split_a(*_fl(_LEFT)), red)
    for q in _SHORT_BOX:
        s.add(_split_a(*_fl(q)), white)
    for q in _TALL_BOX:
        s.add(_split_b(*_fl(q)), white)
    return s


ROUGHNESS_SWEEP = (0.0, 0.05, 0.1, 0.3, 0.5, 0.8)  # modified_cornell.cc:14 (std::vector<float>)


def modified_cornell(roughness: float, res: Tuple[int, int] = (1024, 1024)) -> Scene:
    """examples/modified_cornell.cc: specular room shell with a front wall, 34 triangles."""
    light = Material.make(EMIT, 0, 1, 0)
    red = Material.make(DIFFUSE, (1, 0, 0), 0, 0)
    green = Material.make(DIFFUSE, (0, 1, 0), 0, 0)
    spec = Material.make(SPECULAR, 1, 0, roughness)
    s = Scene(f"modified_cornell_r{roughness}",
              CameraSpec((100.0, 400.0, 0.0), (0.5, -0.5, 1.0), (0.0, 1.0, 0.0), tuple(res), 80.0, 1.0))
    s.add(_split_a(*_fl(_FLOOR)), spec)
    s.add(_split_a(*_fl(_LIGHT)), light)
    s.add(_split_a(*_fl(_CEIL)), spec)
    s.add(_split_a(*_fl(_BACK)), spec)
    s.add(_split_a(*_fl(_FRONT)), spec)
    s.add(_split_a(*_fl(_RIGHT)), spec)
    s.add(_split_a(*_fl(_LEFT)), spec)
    for q in _SHORT_BOX:
        s.add(_split_a(*_fl(q)), red)
    for q in _TALL_BOX:
        s.add(_split_b(*_fl(q)), green)
    return s


def tri3(res: Tuple[int, int] = (512, 512)) -> Scene:
    """tests/test_render.cc: three triangles meeting at the origin, one emissive."""
    s = Scene("tri3", CameraSpec((1.8, 1.8, 1.8), (-1.0, -1.0, -1.0), (0.0, 1.0, 0.0), tuple(res), 60.0, 1.0))
    o, x, y, z = (0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0)
    s.add([(o, x, y)], Material.make(DIFFUSE, (1, 1, 1), 0, 0))
    s.add([(o, z, y)], Material.make(DIFFUSE, (0, 1, 0), 0, 0))
    s.add([(o, x, z)], Material.make(EMIT, (0, 0, 1), 1, 0))
    return s


def sphere_in_cornell(stacks: int = 223, res: Tuple[int, int] = (1024, 1024)) -> Scene:
    """Config 4 stand-in mesh: a UV sphere (stacks x stacks grid, pole fans
    without degenerate triangles) of grey DIFFUSE(0.8), centre (278,200,300),
    radius 120, inside the Cornell box. stacks=223 gives 99,012 sphere + 32 box
    = 99,044 triangles. Vertex coordinates
    are float32-rounded once here so every consumer sees the same values."""
    import numpy as np
    s = cornell(res)
    s.name = f"sphere{stacks}_in_cornell"
    grey = Material.make(DIFFUSE, 0.8, 0, 0)
    cx, cy, cz, rad = 278.0, 200.0, 300.0, 120.0
    slices = stacks
    pts = {}
    for i in range(stacks + 1):
        th = math.pi * i / stacks
        for j in range(slices):
            ph = 2 * math.pi * j / slices
            p = (cx + rad * math.sin(th) * math.cos(ph), cy + rad * math.cos(th),
                 cz + rad * math.sin(th) * math.sin(ph))
            pts[(i, j)] = tuple(float(np.float32(c)) for c in p)
    tris = []
    for i in range(stacks):
        for j in range(slices):
            a, b = pts[(i, j)], pts[(i, (j + 1) % slices)]
            c, d = pts[(i + 1, j)], pts[(i + 1, (j + 1) % slices)]
            if i != 0:
                tris.append((a, c, b))
            if i != stacks - 1:
                tris.append((b, c, d))
    s.add(tris, grey)
    return s


SCENES = {
    "cornell": cornell,
    "tri3": tri3,
}
