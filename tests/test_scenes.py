"""Host-side checks of the procedural stand-in scenes: the arrays are
in the reference Vertex layout (stdafx.h:36-42), inside the unit box, with unit
face normals, and the vectorised ArrayScene path emits exactly what the
per-triangle Scene path emits for the same triangles."""
import numpy as np

from vct import VERTEX_FLOATS, scenes


def _check_arrays(v, i, m, k):
    assert v.dtype == np.float32 and v.shape[1] == VERTEX_FLOATS
    assert i.dtype == np.uint32 and i.size % 3 == 0 and int(i.max()) < v.shape[0]
    assert m.size == i.size // 3 and int(m.max()) < k.shape[0]
    assert np.all(np.abs(v[:, :3]) <= 1.0 + 1e-6)
    nl = np.linalg.norm(v[:, 3:6].astype(np.float64), axis=-1)
    assert np.all(np.abs(nl - 1) < 1e-5)


def test_courtyard_is_san_miguel_class():
    s = scenes.courtyard()
    v, i, m, k = s.arrays()
    _check_arrays(v, i, m, k)
    assert s.n_tri > 1_000_000          # "San Miguel-class": ~1 M triangles, most of them small
    # deterministic (seeded)
    v2, _, m2, _ = scenes.courtyard().arrays()
    assert np.array_equal(v, v2) and np.array_equal(m, m2)


def test_array_scene_matches_list_scene():
    rng = np.random.default_rng(1)
    P = rng.uniform(-0.9, 0.9, (50, 3, 3))
    a, b = scenes.Scene("l"), scenes.ArrayScene("a")
    for s in (a, b):
        s.material((0.5, 0.4, 0.3))
        s.material((0.1, 0.2, 0.3))
    for t in range(50):
        a.tri(P[t, 0], P[t, 1], P[t, 2], t % 2)
    b.tris(P, np.arange(50) % 2)
    for x, y in zip(a.arrays(), b.arrays()):
        assert np.array_equal(x, y)


def test_courtyard_voxelizes_in_oracle(oracle_mod):
    s = scenes.courtyard()
    v, i, m, k = s.arrays()
    n = 32
    g0, E = scenes.grid_for_unit_box(n)
    r = oracle_mod.pipeline(n, g0, E, v, i, m, k, scenes.LIGHT_DIR)
    occ = r["counts"] > 0
    assert occ.sum() > n * n * 3            # floor + three walls at least
    assert (r["r0"][..., :3].sum(-1) > 0).sum() > n * n // 2   # open sky: the paving is lit
