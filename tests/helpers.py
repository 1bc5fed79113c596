"""Shared helpers for the parity tests (test infrastructure)."""
from __future__ import annotations

import numpy as np


def rel_l2(a: np.ndarray, b: np.ndarray) -> float:
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    den = np.linalg.norm(b)
    num = np.linalg.norm(a - b)
    return float(num / den) if den > 0 else float(num)


def scene_arrays(name: str, n_tri: int = 300, seed: int = 7):
    from vct import scenes
    if name == "random":
        s = scenes.random_triangles(n_tri, seed)
    else:
        s = scenes.SCENES[name]()
    return s, s.arrays()


def gpu_pipeline(n, name="cornell", aniso=True, n_diffuse=9, specular=True, light=None, seed=7):
    """K1 -> K2 -> K3 on the GPU through the C-ABI.  -> (ctx, scene, arrays, grid)"""
    from vct import Context, scenes
    s, (v, i, m, k) = scene_arrays(name, seed=seed)
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E, aniso=aniso, n_diffuse=n_diffuse, specular=specular)
    ctx.voxelize(v, i, m, k)
    ctx.inject_directional(light or scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ctx.build_mips()
    return ctx, s, (v, i, m, k), (g0, E)


def gpu_pyramid_flat(ctx) -> np.ndarray:
    """GPU levels 1..L in the oracle's flat layout."""
    parts = []
    for l in range(1, ctx.num_levels):
        _, nf = ctx.level_dims(l)
        for f in range(nf):
            parts.append(ctx.download_level(l, f).ravel())
    return np.concatenate(parts) if parts else np.zeros(0, np.float32)


def write_obj(scene, directory, name="scene"):
    """Wavefront OBJ + MTL of a vct.scenes.Scene (one `usemtl` group per material,
    9-digit floats: float32 positions round-trip exactly).  -> path of the .obj"""
    import os
    v, i, m, k = scene.arrays()
    tri = i.reshape(-1, 3)
    lines = [f"mtllib {name}.mtl"]
    for row in v:
        lines.append("v %.9g %.9g %.9g" % (row[0], row[1], row[2]))
    for mat in range(k.shape[0]):
        sel = np.flatnonzero(m == mat)
        if sel.size == 0:
            continue
        lines.append(f"usemtl m{mat}")
        for t in sel:
            a, b, c = tri[t] + 1
            lines.append(f"f {a} {b} {c}")
    with open(os.path.join(directory, f"{name}.obj"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(directory, f"{name}.mtl"), "w") as f:
        for mat in range(k.shape[0]):
            f.write(f"newmtl m{mat}\nKd %.9g %.9g %.9g\n\n" % tuple(k[mat, :3]))
    return os.path.join(directory, f"{name}.obj")
