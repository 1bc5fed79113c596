"""Row f3: composite + present, CPU side.

The oracle's vo_composite is pinned by closed forms: with an empty grid the
shadow walk always escapes, so final = albedo*color*max(n.l,0) + albedo*diffuse
+ spec exactly (same binary32 operation order); a voxel wall between the point
and the light zeroes the direct term; background pixels are the reference's
clear colour (r_voxelization.cpp:8).  The GPU kernel is compared with the
oracle in tests/test_parity_gpu.py.
"""
import numpy as np


def _frame(rng, h, w, n, g0, E):
    pos = np.zeros((h, w, 4), np.float32)
    pos[..., :3] = rng.uniform(g0[0] + 0.2 * E, g0[0] + 0.8 * E, (h, w, 3))
    pos[..., 3] = (rng.random((h, w)) < 0.8).astype(np.float32)
    nrm = np.zeros((h, w, 4), np.float32)
    v = rng.normal(size=(h, w, 3))
    nrm[..., :3] = v / np.linalg.norm(v, axis=-1, keepdims=True)
    alb = rng.random((h, w, 4)).astype(np.float32)
    dif = rng.random((h, w, 4)).astype(np.float32)
    spe = rng.random((h, w, 4)).astype(np.float32) * 0.2
    return pos, nrm, alb, dif, spe


def _tone(f):
    v = f / (np.float32(1) + f)
    v = np.power(np.maximum(v, np.float32(0)), np.float32(0.454545468), dtype=np.float32)
    return np.clip(np.floor(v.astype(np.float64) * 255.0 + 0.5), 0, 255).astype(np.int64)


def test_composite_empty_grid_closed_form(oracle_mod):
    O = oracle_mod
    n, g0, E = 16, np.array([-1, -1, -1], np.float32), 2.0
    rng = np.random.default_rng(1)
    pos, nrm, alb, dif, spe = _frame(rng, 12, 10, n, g0, E)
    l = np.array([0.3, 1.0, 0.2], np.float32)
    col = np.array([1.0, 0.9, 0.8], np.float32)
    lin, rgba = O.composite(n, g0, E, np.zeros((n, n, n, 4), np.float32), pos, nrm, alb, dif, spe, l, col)
    ln = l / np.sqrt(np.float32((l[0] * l[0] + l[1] * l[1]) + l[2] * l[2]))
    ndl = (nrm[..., 0] * ln[0] + nrm[..., 1] * ln[1]) + nrm[..., 2] * ln[2]
    direct = ((alb[..., :3] * col) * np.maximum(ndl, 0)[..., None]).astype(np.float32)
    exp = (direct + alb[..., :3] * dif[..., :3]) + spe[..., :3]
    valid = pos[..., 3] != 0
    assert np.array_equal(lin[valid][:, :3], exp[valid])
    assert np.all(lin[valid][:, 3] == 1.0)
    assert np.allclose(lin[~valid], [0.2, 0.3, 0.3, 0.0])
    bg = rgba[~valid]
    assert np.all(bg == (51 | (77 << 8) | (77 << 16) | (255 << 24)))
    chans = np.stack([(rgba >> s) & 255 for s in (0, 8, 16)], -1).astype(np.int64)
    assert np.abs(chans[valid] - _tone(exp[valid])).max() <= 1
    assert np.all((rgba >> 24) == 255)


def test_composite_shadowed_by_wall(oracle_mod):
    O = oracle_mod
    n, g0, E = 16, np.array([0, 0, 0], np.float32), 16.0      # 1 voxel = 1 unit
    occ = np.zeros((n, n, n, 4), np.float32)
    occ[12, :, :, 3] = 1.0                                    # wall at z = 12 (index [z][y][x])
    pos = np.zeros((1, 2, 4), np.float32)
    pos[0, 0] = (8.5, 8.5, 4.5, 1.0)                          # below the wall
    pos[0, 1] = (8.5, 8.5, 14.5, 1.0)                         # above it
    nrm = np.zeros((1, 2, 4), np.float32)
    nrm[..., 2] = 1.0
    alb = np.full((1, 2, 4), 0.5, np.float32)
    z = np.zeros((1, 2, 4), np.float32)
    lin, _ = O.composite(n, g0, E, occ, pos, nrm, alb, z, z, (0, 0, 1))
    assert np.all(lin[0, 0, :3] == 0.0)                       # light blocked by the wall
    assert np.all(lin[0, 1, :3] == 0.5)                       # albedo * 1 * n.l = 0.5
