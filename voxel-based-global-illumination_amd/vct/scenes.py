"""Synthetic scenes and G-buffers.

Sponza, San Miguel and the reference's nanosuit.obj are not available offline
(SURVEY.md 0, 8c), so the configs run on procedural stand-ins at the same grid
and framebuffer sizes:

* ``cornell()``: the unit Cornell box [-1,1]^3 without its front face, red left
  wall, green right wall, a short and a tall box; the ceiling has a skylight
  opening so the canonical directional light normalize(0.3, 1, 0.2) reaches the
  interior (with a closed ceiling every voxel would be in shadow);
* ``atrium()``: the "Sponza-class" stand-in: an atrium with a long roof
  opening, two colonnades of four columns, two gallery slabs, coloured walls;
* ``courtyard()``: the "San Miguel-class" stand-in (config C5): an open
  courtyard of 1.0 M mostly small triangles (tessellated paving and walls,
  arcades, icosphere tree crowns, tables, hanging foliage);
* ``random_triangles()``: a triangle soup for voxelization stress / parity;
* ``showroom()``: a textured scene on the reference's own materials
  (assets/model/test/nanosuit.mtl: Arm, Body, Glass, Hand, Helmet, Leg, each
  Kd 0.64 with a map_Kd diffuse map), with TexCoords that repeat (|uv| > 1),
  go negative and vary per face, for the diffuse-map row (albedo = Kd x map).

Geometry is emitted in the reference ``Vertex`` layout (include/stdafx.h:36-42:
Position, Normal, TexCoords, Tangent, Bitangent = 14 floats = 56 bytes,
attribute offsets as mesh.cpp:43-55), uint32 triangle indices, a per-triangle
material index and a Kd table (scene/material.h:10).

G-buffers: ``G_scene`` comes from the HIP ray caster (vct_gbuffer_raycast_device)
or, for small CPU-side fixtures, :func:`raycast_numpy`; ``G_rand`` is
:func:`gbuffer_rand` (positions on occupied voxel centres, jittered voxel
normals, roughness U[0.05, 0.3]; seed 42).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import VERTEX_FLOATS

LIGHT_DIR = (0.3, 1.0, 0.2)      # dir_to_light, SURVEY 8d (normalised by vct_inject_directional)
LIGHT_COLOR = (1.0, 1.0, 1.0)
ROUGHNESS = 0.1                  # G_scene roughness everywhere


def grid_for_unit_box(n: int):
    """Grid AABB = [-1,1]^3 padded by one voxel: E = 2n/(n-2), centred on 0."""
    extent = 2.0 * n / (n - 2)
    return (-extent / 2, -extent / 2, -extent / 2), extent


@dataclass
class Scene:
    name: str
    verts: list = field(default_factory=list)   # rows of 14 floats
    idx: list = field(default_factory=list)
    tri_mat: list = field(default_factory=list)
    kd: list = field(default_factory=list)      # rgba rows
    maps: list = field(default_factory=list)    # per material: diffuse map file name (map_Kd) or None

    def material(self, rgb, diffuse_map: str | None = None) -> int:
        self.kd.append((float(rgb[0]), float(rgb[1]), float(rgb[2]), 1.0))
        self.maps.append(diffuse_map)
        return len(self.kd) - 1

    def material_map(self, names) -> np.ndarray:
        """material_map of vct_voxelize_textured for a texture list in `names` order."""
        return np.array([names.index(m) if m in names else -1 for m in self.maps], np.int32)

    def tri(self, p0, p1, p2, mat: int, uv=None):
        """uv: three (u, v) TexCoords (stored as given: already in the flipped convention)."""
        p0, p1, p2 = (np.asarray(p, np.float64) for p in (p0, p1, p2))
        n = np.cross(p1 - p0, p2 - p0)
        ln = np.linalg.norm(n)
        n = n / ln if ln > 0 else n
        base = len(self.verts)
        for k, p in enumerate((p0, p1, p2)):
            t = (0.0, 0.0) if uv is None else (float(uv[k][0]), float(uv[k][1]))
            self.verts.append([p[0], p[1], p[2], n[0], n[1], n[2], t[0], t[1]] + [0.0] * (VERTEX_FLOATS - 8))
        self.idx += [base, base + 1, base + 2]
        self.tri_mat.append(mat)

    def quad(self, p0, p1, p2, p3, normal, mat: int, uv=None):
        """Quad p0..p3 (in order around the edge) whose face normal points along `normal`;
        uv: the four corners' TexCoords."""
        p0, p1, p2, p3 = (np.asarray(p, np.float64) for p in (p0, p1, p2, p3))
        uv = [(0, 0), (1, 0), (1, 1), (0, 1)] if uv is None else list(uv)
        if np.dot(np.cross(p1 - p0, p2 - p0), normal) < 0:
            p1, p3 = p3, p1
            uv = [uv[0], uv[3], uv[2], uv[1]]
        self.tri(p0, p1, p2, mat, (uv[0], uv[1], uv[2]))
        self.tri(p0, p2, p3, mat, (uv[0], uv[2], uv[3]))

    def box(self, lo, hi, mat: int):
        """Axis-aligned box with outward normals."""
        x0, y0, z0 = lo
        x1, y1, z1 = hi
        self.quad((x0, y0, z0), (x0, y1, z0), (x0, y1, z1), (x0, y0, z1), (-1, 0, 0), mat)
        self.quad((x1, y0, z0), (x1, y1, z0), (x1, y1, z1), (x1, y0, z1), (1, 0, 0), mat)
        self.quad((x0, y0, z0), (x1, y0, z0), (x1, y0, z1), (x0, y0, z1), (0, -1, 0), mat)
        self.quad((x0, y1, z0), (x1, y1, z0), (x1, y1, z1), (x0, y1, z1), (0, 1, 0), mat)
        self.quad((x0, y0, z0), (x1, y0, z0), (x1, y1, z0), (x0, y1, z0), (0, 0, -1), mat)
        self.quad((x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1), (0, 0, 1), mat)

    def rect_y(self, y, x0, x1, z0, z1, ny, mat):
        self.quad((x0, y, z0), (x1, y, z0), (x1, y, z1), (x0, y, z1), (0, ny, 0), mat)

    def arrays(self):
        """(verts (V,14) f32, idx (3T,) u32, tri_mat (T,) u32, kd (M,4) f32)"""
        return (np.asarray(self.verts, np.float32).reshape(-1, VERTEX_FLOATS),
                np.asarray(self.idx, np.uint32),
                np.asarray(self.tri_mat, np.uint32),
                np.asarray(self.kd, np.float32).reshape(-1, 4))

    @property
    def n_tri(self):
        return len(self.tri_mat)


def _ceiling_with_hole(s: Scene, hx0, hx1, hz0, hz1, mat):
    """Ceiling y = 1 (normal -y) with a rectangular skylight [hx0,hx1] x [hz0,hz1]."""
    s.rect_y(1.0, -1.0, 1.0, -1.0, hz0, -1, mat)
    s.rect_y(1.0, -1.0, 1.0, hz1, 1.0, -1, mat)
    s.rect_y(1.0, -1.0, hx0, hz0, hz1, -1, mat)
    s.rect_y(1.0, hx1, 1.0, hz0, hz1, -1, mat)


def cornell() -> Scene:
    s = Scene("cornell")
    white = s.material((0.725, 0.71, 0.68))
    red = s.material((0.63, 0.065, 0.05))
    green = s.material((0.14, 0.45, 0.091))
    s.rect_y(-1.0, -1.0, 1.0, -1.0, 1.0, 1, white)                                   # floor
    _ceiling_with_hole(s, -0.5, 0.5, -0.5, 0.5, white)                               # ceiling
    s.quad((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1), (0, 0, 1), white)     # back
    s.quad((-1, -1, -1), (-1, 1, -1), (-1, 1, 1), (-1, -1, 1), (1, 0, 0), red)       # left
    s.quad((1, -1, -1), (1, 1, -1), (1, 1, 1), (1, -1, 1), (-1, 0, 0), green)        # right
    s.box((0.05, -1.0, 0.0), (0.65, -0.4, 0.6), white)                               # short box
    s.box((-0.65, -1.0, -0.6), (-0.05, 0.2, 0.0), white)                             # tall box
    return s


def atrium() -> Scene:
    """Sponza-class stand-in: atrium with colonnades, galleries and a roof opening."""
    s = Scene("atrium")
    stone = s.material((0.72, 0.68, 0.60))
    floor = s.material((0.55, 0.50, 0.45))
    red = s.material((0.60, 0.12, 0.10))
    blue = s.material((0.12, 0.20, 0.55))
    green = s.material((0.20, 0.45, 0.15))
    ochre = s.material((0.75, 0.55, 0.20))
    s.rect_y(-1.0, -1.0, 1.0, -1.0, 1.0, 1, floor)
    _ceiling_with_hole(s, -0.35, 0.35, -0.85, 0.85, stone)
    s.quad((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1), (0, 0, 1), ochre)
    s.quad((-1, -1, -1), (-1, 1, -1), (-1, 1, 1), (-1, -1, 1), (1, 0, 0), red)
    s.quad((1, -1, -1), (1, 1, -1), (1, 1, 1), (1, -1, 1), (-1, 0, 0), blue)
    # two gallery slabs along the side walls at mid height
    s.box((-1.0, 0.05, -1.0), (-0.55, 0.15, 0.8), stone)
    s.box((0.55, 0.05, -1.0), (1.0, 0.15, 0.8), stone)
    # colonnades: 4 columns per side (ground floor) + 4 per side (gallery level)
    for side in (-1, 1):
        x = side * 0.5
        for k in range(4):
            z = -0.8 + k * 0.5
            s.box((x - 0.06, -1.0, z - 0.06), (x + 0.06, 0.05, z + 0.06), stone)
            s.box((x - 0.045, 0.15, z - 0.045), (x + 0.045, 0.85, z + 0.045), stone)
        # balustrade on the gallery edge
        s.box((x - 0.03, 0.15, -0.95), (x + 0.03, 0.3, 0.75), green)
    # a fountain block in the middle of the court
    s.box((-0.2, -1.0, -0.2), (0.2, -0.8, 0.2), stone)
    return s


def random_triangles(n_tri: int, seed: int = 7, size: float = 0.3) -> Scene:
    """Triangle soup inside [-1,1]^3 (sizes up to `size`), random materials."""
    rng = np.random.default_rng(seed)
    s = Scene("random")
    mats = [s.material(rng.uniform(0.05, 0.95, 3)) for _ in range(5)]
    c = rng.uniform(-0.9, 0.9, (n_tri, 3))
    for t in range(n_tri):
        p = c[t] + rng.uniform(-size, size, (3, 3))
        s.tri(p[0], p[1], p[2], mats[t % len(mats)])
    return s


class ArrayScene(Scene):
    """A scene built directly as arrays (for million-triangle stand-ins, where the
    per-triangle list path of :class:`Scene` would be slow).  Triangles are added in
    batches with the same per-corner vertex rule as :meth:`Scene.tri` (flat face
    normal, computed in float64, stored as float32)."""

    def __init__(self, name: str):
        super().__init__(name)
        self._pos: list = []      # (T,3,3) float64 batches
        self._mat: list = []      # (T,) int batches

    def tris(self, P: np.ndarray, mat) -> None:
        P = np.asarray(P, np.float64).reshape(-1, 3, 3)
        self._pos.append(P)
        self._mat.append(np.broadcast_to(np.asarray(mat, np.int64), (P.shape[0],)).copy())

    def tri(self, p0, p1, p2, mat: int):
        self.tris(np.stack([np.asarray(p, np.float64) for p in (p0, p1, p2)])[None], mat)

    def arrays(self):
        P = np.concatenate(self._pos) if self._pos else np.zeros((0, 3, 3))
        mat = np.concatenate(self._mat) if self._mat else np.zeros((0,), np.int64)
        n = np.cross(P[:, 1] - P[:, 0], P[:, 2] - P[:, 0])
        ln = np.linalg.norm(n, axis=-1, keepdims=True)
        n = np.where(ln > 0, n / np.where(ln > 0, ln, 1.0), n)
        T = P.shape[0]
        verts = np.zeros((T, 3, VERTEX_FLOATS), np.float32)
        verts[:, :, 0:3] = P
        verts[:, :, 3:6] = n[:, None, :]
        return (verts.reshape(-1, VERTEX_FLOATS), np.arange(3 * T, dtype=np.uint32),
                mat.astype(np.uint32), np.asarray(self.kd, np.float32).reshape(-1, 4))

    @property
    def n_tri(self):
        return int(sum(p.shape[0] for p in self._pos))


def _grid_quads(xs, zs, y):
    """Heightfield y(x,z) over the grid xs x zs -> (2*(nx-1)*(nz-1), 3, 3) triangles
    wound so the face normal points up."""
    X, Z = np.meshgrid(xs, zs, indexing="xy")
    Y = y(X, Z)
    V = np.stack([X, Y, Z], -1)
    a, b = V[:-1, :-1], V[:-1, 1:]
    c, d = V[1:, 1:], V[1:, :-1]
    t1 = np.stack([a, d, c], -2).reshape(-1, 3, 3)
    t2 = np.stack([a, c, b], -2).reshape(-1, 3, 3)
    return np.concatenate([t1, t2])


def _orient(T: np.ndarray, normal) -> np.ndarray:
    """Reverse the winding of the triangles whose face normal opposes `normal`."""
    fn = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
    flip = fn @ np.asarray(normal, np.float64) < 0
    T = T.copy()
    T[flip] = T[flip][:, ::-1]
    return T


def _icosphere(level: int):
    """Unit icosphere triangles (20 * 4^level, 3, 3), outward winding."""
    t = (1 + 5 ** 0.5) / 2
    v = np.array([(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
                  (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)], np.float64)
    f = np.array([(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2),
                  (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5),
                  (2, 4, 11), (6, 2, 10), (8, 6, 7), (9, 8, 1)])
    T = v[f]
    T /= np.linalg.norm(T, axis=-1, keepdims=True)
    for _ in range(level):
        a, b, c = T[:, 0], T[:, 1], T[:, 2]
        ab, bc, ca = (a + b) / 2, (b + c) / 2, (c + a) / 2
        ab, bc, ca = (x / np.linalg.norm(x, axis=-1, keepdims=True) for x in (ab, bc, ca))
        T = np.concatenate([np.stack(q, 1) for q in ((a, ab, ca), (ab, b, bc), (ca, bc, c), (ab, bc, ca))])
    return T


def _box_tris(lo, hi):
    s = Scene("tmp")
    s.box(lo, hi, 0)
    return np.asarray(s.verts, np.float64)[:, :3].reshape(-1, 3, 3)


def courtyard(seed: int = 11) -> Scene:
    """"San Miguel-class" stand-in (BASELINE config C5): an open courtyard with
    ~1.1 M triangles, most of them small: a finely tessellated undulating paving
    (the bulk of the count), arcaded walls, tessellated tree crowns on trunks,
    tables, and a hanging-foliage triangle soup along the upper arcade."""
    rng = np.random.default_rng(seed)
    s = ArrayScene("courtyard")
    paving = s.material((0.60, 0.52, 0.42))
    plaster = s.material((0.78, 0.70, 0.55))
    terracotta = s.material((0.65, 0.30, 0.18))
    bark = s.material((0.35, 0.25, 0.15))
    leaves = s.material((0.18, 0.42, 0.12))
    wood = s.material((0.50, 0.33, 0.20))
    # paving: 600 x 600 quads, gentle undulation (720 K triangles)
    xs = np.linspace(-1.0, 1.0, 601)
    s.tris(_grid_quads(xs, xs, lambda X, Z: -0.985 + 0.015 * np.sin(7 * X) * np.cos(5 * Z)), paving)
    # walls (back, left, right), tessellated 120 x 120 each (86 K triangles)
    ws = np.linspace(-1.0, 1.0, 121)
    wall = _grid_quads(ws, ws, lambda X, Z: np.zeros_like(X))    # (a, 0, b) grid
    a, b = wall[..., 0], wall[..., 2]
    one = np.ones_like(a)
    s.tris(_orient(np.stack([a, b, -one], -1), (0, 0, 1)), plaster)       # back  z = -1, normal +z
    s.tris(_orient(np.stack([-one, a, b], -1), (1, 0, 0)), terracotta)    # left  x = -1, normal +x
    s.tris(_orient(np.stack([one, a, b], -1), (-1, 0, 0)), terracotta)    # right x = +1, normal -x
    # arcade: piers and an upper gallery slab along the three walls
    for k in range(7):
        z = -0.9 + k * 0.3
        s.tris(_box_tris((-0.86, -1.0, z - 0.04), (-0.78, 0.1, z + 0.04)), plaster)
        s.tris(_box_tris((0.78, -1.0, z - 0.04), (0.86, 0.1, z + 0.04)), plaster)
    for k in range(6):
        x = -0.75 + k * 0.3
        s.tris(_box_tris((x - 0.04, -1.0, -0.86), (x + 0.04, 0.1, -0.78)), plaster)
    s.tris(_box_tris((-1.0, 0.1, -1.0), (-0.75, 0.18, 0.95)), plaster)
    s.tris(_box_tris((0.75, 0.1, -1.0), (1.0, 0.18, 0.95)), plaster)
    s.tris(_box_tris((-0.75, 0.1, -1.0), (0.75, 0.18, -0.75)), plaster)
    # trees: trunks + icosphere crowns (level 4: 5120 triangles each)
    crown = _icosphere(4)
    for (tx, tz, r) in ((-0.4, -0.3, 0.22), (0.35, -0.45, 0.25), (0.05, 0.3, 0.18), (-0.45, 0.45, 0.16),
                        (0.5, 0.35, 0.2)):
        top = -0.35 + r
        s.tris(_box_tris((tx - 0.025, -1.0, tz - 0.025), (tx + 0.025, top - r * 0.5, tz + 0.025)), bark)
        for j in range(3):
            off = rng.uniform(-0.5, 0.5, 3) * r
            s.tris(crown * (r * rng.uniform(0.6, 0.9)) + np.array([tx, top, tz]) + off, leaves)
    # tables with tops and legs (dining area)
    for k in range(24):
        cx, cz = rng.uniform(-0.65, 0.65), rng.uniform(-0.65, 0.75)
        s.tris(_box_tris((cx - 0.07, -0.78, cz - 0.07), (cx + 0.07, -0.76, cz + 0.07)), wood)
        for dx in (-0.05, 0.05):
            for dz in (-0.05, 0.05):
                s.tris(_box_tris((cx + dx - 0.006, -1.0, cz + dz - 0.006), (cx + dx + 0.006, -0.78, cz + dz + 0.006)),
                       wood)
    # hanging foliage on the gallery edge: 120 K small triangles
    nf = 120_000
    side = rng.integers(0, 3, nf)
    u = rng.uniform(-0.95, 0.95, nf)
    yy = rng.uniform(-0.35, 0.1, nf)
    c = np.where(side[:, None] == 0, np.stack([np.full(nf, -0.74), yy, u], -1),
                 np.where(side[:, None] == 1, np.stack([np.full(nf, 0.74), yy, u], -1),
                          np.stack([u * 0.78, yy, np.full(nf, -0.74)], -1)))
    c += rng.uniform(-0.03, 0.03, c.shape)
    s.tris(c[:, None, :] + rng.uniform(-0.012, 0.012, (nf, 3, 3)), leaves)
    return s


# the reference's material library, assets/model/test/nanosuit.mtl:3-77 (name, map_Kd; Kd 0.64)
NANOSUIT_MATERIALS = (("Arm", "arm_dif.png"), ("Body", "body_dif.png"), ("Glass", "glass_dif.png"),
                      ("Hand", "hand_dif.png"), ("Helmet", "helmet_diff.png"), ("Leg", "leg_dif.png"))
NANOSUIT_KD = 0.64


def showroom(sphere_level: int = 2) -> Scene:
    """Textured stand-in on nanosuit.mtl's materials: a floor with tiled UVs (x3,
    GL_REPEAT), back / side walls with negative and offset UVs, a plinth box per
    material with per-face [0,1]^2 UVs, and a spherical-UV icosphere (the seam makes
    some triangles span u in [0.9, 1.1])."""
    s = Scene("showroom")
    m = {name: s.material((NANOSUIT_KD,) * 3, path) for name, path in NANOSUIT_MATERIALS}
    plain = s.material((0.5, 0.45, 0.4))                                     # an unmapped material
    s.rect_y(-1.0, -1.0, 1.0, -1.0, 1.0, 1, m["Leg"])
    s.quad((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1), (0, 0, 1), m["Body"],
           uv=[(0, 0), (3, 0), (3, 3), (0, 3)])                                   # floor-like tiling on the back wall
    s.quad((-1, -1, -1), (-1, 1, -1), (-1, 1, 1), (-1, -1, 1), (1, 0, 0), m["Arm"],
           uv=[(-0.5, -0.25), (-0.5, 1.75), (1.5, 1.75), (1.5, -0.25)])          # negative UVs
    s.quad((1, -1, -1), (1, 1, -1), (1, 1, 1), (1, -1, 1), (-1, 0, 0), plain)
    for k, name in enumerate(("Hand", "Glass", "Helmet")):
        x = -0.6 + 0.6 * k
        lo, hi = np.array([x - 0.2, -1.0, -0.5]), np.array([x + 0.2, -0.55 + 0.15 * k, -0.1])
        _box_uv(s, lo, hi, m[name])
    T = _icosphere(sphere_level) * 0.3 + np.array([0.0, 0.2, 0.35])
    for tri in T:
        d = (tri - np.array([0.0, 0.2, 0.35])) / 0.3
        u = 0.5 + np.arctan2(d[:, 2], d[:, 0]) / (2 * np.pi)
        u = np.where(u - u.min() > 0.5, u - 1.0, u)                           # seam: keep a triangle's u contiguous
        v = 0.5 - np.arcsin(np.clip(d[:, 1], -1, 1)) / np.pi
        s.tri(tri[0], tri[1], tri[2], m["Helmet"], uv=list(zip(u, v)))
    return s


def _box_uv(s: Scene, lo, hi, mat):
    """Axis-aligned box with outward normals and [0,1]^2 TexCoords per face."""
    x0, y0, z0 = lo
    x1, y1, z1 = hi
    s.quad((x0, y0, z0), (x0, y1, z0), (x0, y1, z1), (x0, y0, z1), (-1, 0, 0), mat)
    s.quad((x1, y0, z0), (x1, y1, z0), (x1, y1, z1), (x1, y0, z1), (1, 0, 0), mat)
    s.quad((x0, y0, z0), (x1, y0, z0), (x1, y0, z1), (x0, y0, z1), (0, -1, 0), mat)
    s.quad((x0, y1, z0), (x1, y1, z0), (x1, y1, z1), (x0, y1, z1), (0, 1, 0), mat)
    s.quad((x0, y0, z0), (x1, y0, z0), (x1, y1, z0), (x0, y1, z0), (0, 0, -1), mat)
    s.quad((x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1), (0, 0, 1), mat)


SCENES = {"cornell": cornell, "atrium": atrium, "courtyard": courtyard, "showroom": showroom}


# ---------------------------------------------------------------------------
# G-buffers
# ---------------------------------------------------------------------------

def raycast_numpy(scene: Scene, cam, w: int, h: int, roughness: float = ROUGHNESS):
    """CPU G_scene (same ray rule as the HIP caster; for small fixtures only)."""
    verts, idx, mat, kd = scene.arrays()
    P = verts[:, :3].astype(np.float64)[idx.reshape(-1, 3)]
    v0, e1, e2 = P[:, 0], P[:, 1] - P[:, 0], P[:, 2] - P[:, 0]
    th = np.tan(np.radians(cam.zoom) / 2)
    aspect = w / h
    xs = (2 * (np.arange(w) + 0.5) / w - 1) * th * aspect
    ys = (1 - 2 * (np.arange(h) + 0.5) / h) * th
    X, Y = np.meshgrid(xs, ys)
    d = cam.front[None, None] + X[..., None] * cam.right + Y[..., None] * cam.up
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    d = d.reshape(-1, 3)
    o = cam.position
    best = np.full(d.shape[0], np.inf)
    hit = np.full(d.shape[0], -1)
    for t in range(len(v0)):
        pv = np.cross(d, e2[t])
        det = pv @ e1[t]
        ok = np.abs(det) >= 1e-12
        inv = np.where(ok, 1.0 / np.where(ok, det, 1.0), 0.0)
        tv = o - v0[t]
        u = (pv @ tv) * inv
        qv = np.cross(tv, e1[t])
        v = (d @ qv) * inv
        tt = (qv @ e2[t]) * inv
        m = ok & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (tt > 0) & (tt < best)
        best[m] = tt[m]
        hit[m] = t
    depth = best * (d @ cam.front)
    valid = (hit >= 0) & (depth >= cam.near) & (depth <= cam.far)
    pos = np.zeros((d.shape[0], 4), np.float32)
    nrm = np.zeros((d.shape[0], 4), np.float32)
    alb = np.zeros((d.shape[0], 4), np.float32)
    alb[:, 3] = roughness
    hv = hit[valid]
    pos[valid, :3] = o + d[valid] * best[valid, None]
    pos[valid, 3] = 1.0
    fn = np.cross(e1[hv], e2[hv])
    fn /= np.linalg.norm(fn, axis=-1, keepdims=True)
    flip = np.einsum("ij,ij->i", fn, d[valid]) > 0
    fn[flip] *= -1
    nrm[valid, :3] = fn
    alb[valid, :3] = kd[mat[hv], :3]
    return pos.reshape(h, w, 4), nrm.reshape(h, w, 4), alb.reshape(h, w, 4)


def gbuffer_rand(albedo_occ: np.ndarray, normal: np.ndarray, aabb_min, extent: float, w: int, h: int,
                 seed: int = 42):
    """G_rand: cache-hostile stress G-buffer on occupied voxel centres."""
    n = albedo_occ.shape[0]
    rng = np.random.default_rng(seed)
    flat_occ = albedo_occ.reshape(-1, 4)[:, 3] > 0
    occ = np.flatnonzero(flat_occ)
    if occ.size == 0:
        raise ValueError("empty voxel grid")
    pick = occ[rng.integers(0, occ.size, w * h)]
    x, y, z = pick % n, (pick // n) % n, pick // (n * n)
    hvox = extent / n
    g0 = np.asarray(aabb_min, np.float64)
    pos = np.ones((w * h, 4), np.float32)
    pos[:, 0] = g0[0] + hvox * (x + 0.5)
    pos[:, 1] = g0[1] + hvox * (y + 0.5)
    pos[:, 2] = g0[2] + hvox * (z + 0.5)
    nv = normal.reshape(-1, 4)[pick, :3].astype(np.float64)
    zero = np.linalg.norm(nv, axis=-1) < 1e-6
    nv[zero] = rng.normal(size=(zero.sum(), 3))
    nv += rng.uniform(-0.1, 0.1, nv.shape)
    nv /= np.linalg.norm(nv, axis=-1, keepdims=True)
    nrm = np.zeros((w * h, 4), np.float32)
    nrm[:, :3] = nv
    alb = np.zeros((w * h, 4), np.float32)
    alb[:, :3] = albedo_occ.reshape(-1, 4)[pick, :3]
    alb[:, 3] = rng.uniform(0.05, 0.3, w * h)
    return pos.reshape(h, w, 4), nrm.reshape(h, w, 4), alb.reshape(h, w, 4)
