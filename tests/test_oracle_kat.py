"""Pins the CPU oracle (oracle/vct_oracle.c) -- CPU only, no GPU.

The reference holds no implementation, test, fixture or golden vector for this
path, so the oracle is pinned two ways:
  1. closed-form known-answer tests of SURVEY.md 8c (KAT 1-5);
  2. bit-for-bit agreement with an independent numpy / pure-Python restatement
     of Appendix A (tests/spec_ref.py) on small inputs.
"""
import math

import numpy as np
import pytest

import spec_ref as R


@pytest.fixture(scope="module")
def O(oracle_mod):
    return oracle_mod


def _scene(name, n):
    from vct import scenes
    s = scenes.random_triangles(60, seed=11) if name == "random" else scenes.SCENES[name]()
    g0, E = scenes.grid_for_unit_box(n)
    return s, s.arrays(), g0, E


# -- log2 -------------------------------------------------------------------
def test_log2_accuracy_and_exact_powers(O):
    xs = np.concatenate([np.linspace(1, 2, 257), np.geomspace(1, 1024, 2000)]).astype(np.float32)
    got = np.array([O.log2(float(x)) for x in xs])
    assert np.max(np.abs(got - np.log2(xs.astype(np.float64)))) < 4e-7 * 11
    for k in range(11):
        assert O.log2(2.0 ** k) == float(k)
    for x in xs[::37]:
        assert O.log2(float(x)) == R.log2(float(x))


# -- KAT 1: empty grid --------------------------------------------------------
def _empty_grid_steps(o, d, tau, n):
    """Closed-form step count of one cone in an empty grid (float32 t-sequence)."""
    f32 = R.f32
    t, steps, tmax = 1.0, 0, f32(f32(n) * R.SQRT3)
    tau2 = f32(2 * tau)
    while t <= tmax:
        q = [f32(o[i] + f32(d[i] * t)) for i in range(3)]
        if not all(0 <= v <= n for v in q):
            break
        D = max(1.0, f32(tau2 * t))
        t = f32(t + f32(0.5 * D))
        steps += 1
    return steps


@pytest.mark.parametrize("aniso", [True, False])
def test_kat1_empty_grid(O, aniso):
    n, E = 32, 2.0
    g0 = (-1.0, -1.0, -1.0)
    r0 = np.zeros((n, n, n, 4), np.float32)
    pyr = O.build_mips(n, r0, aniso)
    assert not pyr.any()
    pos = np.zeros((1, 3, 4), np.float32)
    pos[0, :, :3] = [[0.0, 0.0, 0.0], [0.3, -0.7, 0.2], [-0.9, 0.9, -0.9]]
    pos[..., 3] = 1
    nrm = np.zeros_like(pos)
    nrm[0, 0, :3] = [0, 1, 0]
    nrm[0, 1, :3] = [0, 0, 1]
    nrm[0, 2, :3] = [1, 0, 0]
    alb = np.full_like(pos, 0.1)
    eye = (0.0, 0.0, 3.0)
    res = O.trace(n, g0, E, r0, pyr, pos, nrm, alb, eye, aniso=aniso, n_diffuse=9, specular=True)
    assert not res["diffuse"][..., :3].any() and np.all(res["diffuse"][..., 3] == 1.0)
    assert not res["spec"].any()
    # the step count equals the closed-form count of every cone's t-sequence
    tr = R.Tracer(n, g0, E, r0, {}, aniso)
    for i in range(3):
        P, N = pos[0, i], nrm[0, i]
        o = [R.f32(R.f32(R.f32(float(P[k]) - tr.g0[k]) * tr.inv_h) + float(N[k])) for k in range(3)]
        nx, ny, nz = (float(v) for v in N[:3])
        sgn = math.copysign(1.0, nz)
        ka = R.f32(-1.0 / R.f32(sgn + nz))
        kb = R.f32(R.f32(nx * ny) * ka)
        T = [R.f32(1.0 + R.f32(R.f32(R.f32(sgn * nx) * nx) * ka)), R.f32(sgn * kb), -R.f32(sgn * nx)]
        B = [kb, R.f32(sgn + R.f32(R.f32(ny * ny) * ka)), -ny]
        expect = 0
        for cn, ct, cb, _ in R.CONES9:
            d = [R.f32(R.f32(R.f32(cn * a) + R.f32(ct * b)) + R.f32(cb * c)) for a, b, c in zip((nx, ny, nz), T, B)]
            expect += _empty_grid_steps(o, d, R.TAN30, n)
        v = [R.f32(float(eye[k]) - float(P[k])) for k in range(3)]
        vl = R.f32(math.sqrt(R.f32(R.f32(R.f32(v[0] * v[0]) + R.f32(v[1] * v[1])) + R.f32(v[2] * v[2]))))
        v = [R.f32(x / vl) for x in v]
        ndv = R.f32(R.f32(R.f32(nx * v[0]) + R.f32(ny * v[1])) + R.f32(nz * v[2]))
        r = [R.f32(R.f32(R.f32(2 * ndv) * a) - b) for a, b in zip((nx, ny, nz), v)]
        expect += _empty_grid_steps(o, r, 0.1, n)
        assert res["steps_px"][0, i] == expect


# -- KAT 2: constant level 0 -> a_l = 1 - (1 - alpha)^(2^l) ----------------------
@pytest.mark.parametrize("alpha,L", [(0.3, 0.8), (1.0, 0.25), (0.05, 2.0)])
def test_kat2_constant_mips(O, alpha, L):
    n = 16
    r0 = np.empty((n, n, n, 4), np.float32)
    r0[..., :3] = L * alpha
    r0[..., 3] = alpha
    lv = O.pyramid_levels(n, O.build_mips(n, r0, True), True)
    for l, faces in lv.items():
        al = 1 - (1 - alpha) ** (2 ** l)
        for f in faces:
            np.testing.assert_allclose(f[..., 3], al, rtol=3e-6)
            np.testing.assert_allclose(f[..., :3], L * al, rtol=3e-6)   # premultiplied invariant
    iso = O.pyramid_levels(n, O.build_mips(n, r0, False), False)
    for l, (f,) in iso.items():
        np.testing.assert_allclose(f[..., 3], alpha, rtol=1e-6)


# -- KAT 3: opaque emissive plane ---------------------------------------------
@pytest.mark.parametrize("k", [3, 6, 12])
def test_kat3_plane(O, k):
    """Opaque plane x = x0 of colour Lc; a pixel k voxels in front, normal +x,
    one cone along +x: the cone saturates, c = Lc * a (premultiplied invariant),
    and it stops no earlier than the sample footprint reaches the plane and no
    later than two steps after it."""
    n, E, x0 = 64, 64.0, 40
    g0 = (0.0, 0.0, 0.0)
    Lc = np.array([0.7, 0.4, 0.2], np.float32)
    r0 = np.zeros((n, n, n, 4), np.float32)
    r0[:, :, x0, :3] = Lc
    r0[:, :, x0, 3] = 1
    pyr = O.build_mips(n, r0, True)
    px = x0 - k  # voxel x of the surface point
    pos = np.array([[[px + 0.5 - 1.0, 32.0, 32.0, 1.0]]], np.float32)  # o = P + n lands at px + 0.5
    nrm = np.array([[[1.0, 0.0, 0.0, 0.0]]], np.float32)
    alb = np.full_like(pos, 0.1)
    res = O.trace(n, g0, E, r0, pyr, pos, nrm, alb, (0, 0, 0), n_diffuse=1, specular=False)
    c, ao = res["diffuse"][0, 0, :3], res["diffuse"][0, 0, 3]
    a = 1 - ao
    assert a >= 0.95
    np.testing.assert_allclose(c, Lc * a, rtol=2e-5)
    # replay the t-sequence: the stopping step's footprint [t - D/2, t + D/2] reaches the plane
    dist = x0 - (px + 0.5)
    t, steps, reached = 1.0, 0, None
    while steps < res["steps_px"][0, 0]:
        D = max(1.0, R.f32(R.f32(2 * R.TAN30) * t))
        if reached is None and t + D / 2 + 0.5 >= dist:
            reached = steps + 1
        t = R.f32(t + R.f32(0.5 * D))
        steps += 1
    assert reached is not None and steps >= reached   # never stops before the plane
    # and the exact stopping step equals the independent restatement's
    tr = R.Tracer(n, g0, E, r0, O.pyramid_levels(n, pyr, True), True)
    d, _, st = tr.pixel(pos[0, 0], nrm[0, 0], 0.1, (0, 0, 0), cones=R.CONES1, specular=False)
    assert st == res["steps_px"][0, 0] and np.array_equal(np.float32(d), res["diffuse"][0, 0])


# -- KAT 4: voxelization -------------------------------------------------------
def test_kat4_axis_aligned_quad_slab(O):
    """A z = const quad strictly inside a voxel layer covers exactly that layer's slab."""
    n = 16
    g0, E = (0.0, 0.0, 0.0), 16.0
    z = 5.37
    x0, x1, y0, y1 = 2.3, 9.6, 4.1, 12.9
    v = np.zeros((4, 14), np.float32)
    v[:, :3] = [[x0, y0, z], [x1, y0, z], [x1, y1, z], [x0, y1, z]]
    idx = np.array([0, 1, 2, 0, 2, 3], np.uint32)
    sums, counts = O.voxelize(n, g0, E, v, idx)
    occ = counts.reshape(n, n, n) > 0
    expect = np.zeros((n, n, n), bool)
    expect[5, 4:13, 2:10] = True
    assert np.array_equal(occ, expect)
    # diagonal voxels are hit by both triangles: count 2, the normal sum is 2 * (0,0,1)
    nz = sums.reshape(n, n, n, 6)[..., 5]
    assert np.all(nz[occ] == 65536 * counts.reshape(n, n, n)[occ])


def test_kat4_random_tris_vs_bruteforce(O):
    """Every voxel a brute-force SAT over ALL n^3 voxels accepts is covered, and nothing else."""
    n = 16
    s, (v, i, m, k), g0, E = _scene("random", n)
    sums, counts = O.voxelize(n, g0, E, v, i, m, k)
    zz, yy, xx = np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing="ij")
    c = [a.astype(np.float32) + np.float32(0.5) for a in (xx, yy, zz)]
    inv_h = np.float32(n) / np.float32(E)
    brute = np.zeros(n ** 3, np.int64)
    for tri in i.reshape(-1, 3):
        q = (v[tri, :3].astype(np.float32) - np.asarray(g0, np.float32)) * inv_h
        brute += R._sat(q, *c).ravel()
    assert np.array_equal(brute, counts.astype(np.int64))


# -- KAT 5: injection -----------------------------------------------------------
def test_kat5_injection(O):
    n = 16
    ao = np.zeros((n, n, n, 4), np.float32)
    nm = np.zeros((n, n, n, 4), np.float32)
    ao[8, 8, 8] = (0.5, 0.25, 1.0, 1.0)
    nm[8, 8, 8, :3] = (0, 1, 0)
    ao[3, 3, 3] = (0.5, 0.5, 0.5, 1.0)
    nm[3, 3, 3, :3] = (1, 0, 0)
    color = (2.0, 1.0, 0.5)
    # light perpendicular to the first normal -> 0, cos(theta) = 0 for it
    r0 = O.inject(n, ao, nm, (1.0, 0.0, 0.0), color)
    assert np.all(r0[8, 8, 8, :3] == 0) and r0[8, 8, 8, 3] == 1
    # unoccluded voxel lit at 60 degrees: albedo * color * cos
    l = np.array([0.0, 0.5, math.sqrt(3) / 2])
    r0 = O.inject(n, ao, nm, l, color)
    np.testing.assert_allclose(r0[8, 8, 8, :3], np.array([0.5, 0.25, 1.0]) * np.array(color) * 0.5, rtol=1e-6)
    # an occluder on the light path shadows it
    # (the ray from centre + n = (8.5, 9.5, 8.5) along (0, .5, .866) enters voxel
    # (x, y, z) = (8, 9, 9) then (8, 10, 9); arrays are indexed [z][y][x])
    ao2 = ao.copy()
    ao2[9, 10, 8] = (1, 1, 1, 1)
    r0 = O.inject(n, ao2, nm, l, color)
    assert np.all(r0[8, 8, 8, :3] == 0)
    ao3 = ao.copy()
    ao3[9, 11, 8] = (1, 1, 1, 1)        # off the path: still lit
    r0 = O.inject(n, ao3, nm, l, color)
    assert np.all(r0[8, 8, 8, :3] > 0)
    assert np.all(r0[ao3[..., 3] == 0] == 0) and np.all(r0[ao3[..., 3] != 0][:, 3] == 1)


# -- oracle == independent restatement, bit for bit ------------------------------
@pytest.mark.parametrize("name", ["cornell", "atrium", "random"])
def test_oracle_matches_spec_ref_pipeline(O, name):
    n = 16
    s, (v, i, m, k), g0, E = _scene(name, n)
    sums, counts = O.voxelize(n, g0, E, v, i, m, k)
    rs, rc = R.voxelize(n, g0, E, v, i, m, k)
    assert np.array_equal(counts, rc) and np.array_equal(sums, rs)
    ao, nm = O.resolve(n, sums, counts)
    rao, rnm = R.resolve(n, sums, counts)
    assert np.array_equal(ao, rao) and np.array_equal(nm, rnm)
    from vct import scenes
    r0 = O.inject(n, ao, nm, scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    assert np.array_equal(r0, R.inject(n, ao, nm, scenes.LIGHT_DIR, scenes.LIGHT_COLOR))
    assert r0[..., :3].sum() > 0
    for aniso in (True, False):
        lv = O.pyramid_levels(n, O.build_mips(n, r0, aniso), aniso)
        ref = R.build_mips(r0, aniso)
        for l in lv:
            for f in range(len(lv[l])):
                assert np.array_equal(lv[l][f], ref[l][f]), (aniso, l, f)


@pytest.mark.parametrize("aniso", [True, False])
def test_oracle_matches_spec_ref_trace(O, aniso):
    from vct import scenes
    from vct.camera import Camera
    n = 16
    s, (v, i, m, k), g0, E = _scene("cornell", n)
    st = O.pipeline(n, g0, E, v, i, m, k, scenes.LIGHT_DIR, aniso=aniso)
    cam = Camera()
    pos, nrm, alb = scenes.raycast_numpy(s, cam, 16, 12)
    alb[..., 3] = np.linspace(0.01, 0.5, alb[..., 3].size).reshape(alb.shape[:2])
    res = O.trace(n, g0, E, st["r0"], st["pyr"], pos, nrm, alb, cam.position, aniso=aniso)
    tr = R.Tracer(n, g0, E, st["r0"], O.pyramid_levels(n, st["pyr"], aniso), aniso)
    rng = np.random.default_rng(1)
    valid = np.argwhere(pos[..., 3] != 0)
    for y, x in valid[rng.choice(len(valid), 6, replace=False)]:
        d, sp, steps = tr.pixel(pos[y, x], nrm[y, x], alb[y, x, 3], cam.position)
        assert steps == res["steps_px"][y, x]
        assert np.array_equal(np.float32(d), res["diffuse"][y, x]), (y, x)
        assert np.array_equal(np.float32(sp), res["spec"][y, x]), (y, x)
