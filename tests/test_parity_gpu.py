"""Parity of the HIP path (through the C-ABI) with the CPU oracle.

Bar: K1 voxelization, K2 injection and K3 mips are
integer / fixed-order float work -> BIT-EXACT.  K4 cone tracing: relative L2
<= 1e-3 over both output buffers (north_star's fp32 tolerance); the kernels
and the oracle share the spec's operation order, so the observed error is
expected to be 0 and the per-pixel step counts identical.
"""
import ctypes as C

import numpy as np
import pytest

from helpers import gpu_pipeline, gpu_pyramid_flat, rel_l2, scene_arrays

pytestmark = pytest.mark.gpu

TRACE_TOL = 1e-3   # north_star: indirect-irradiance parity within 1e-3 relative L2 (fp32)


@pytest.mark.parametrize("name,n", [("cornell", 16), ("cornell", 32), ("atrium", 32), ("atrium", 64),
                                    ("random", 32), ("courtyard", 64)])
def test_voxelize_inject_mips_bitexact(gpu_ready, oracle_mod, name, n):
    O = oracle_mod
    ctx, s, (v, i, m, k), (g0, E) = gpu_pipeline(n, name)
    ref = O.pipeline(n, g0, E, v, i, m, k, __import__("vct").scenes.LIGHT_DIR)
    sums, counts = ctx.download_accum()
    assert np.array_equal(counts, ref["counts"]), "K1 coverage counts differ"
    assert np.array_equal(sums, ref["sums"]), "K1 fixed-point sums differ"
    ao, nm = ctx.download_voxels()
    assert np.array_equal(ao, ref["albedo_occ"])
    assert np.array_equal(nm, ref["normal"])
    r0 = ctx.download_level(0)
    assert np.array_equal(r0, ref["r0"]), "K2 radiance differs"
    assert np.array_equal(gpu_pyramid_flat(ctx), ref["pyr"]), "K3 pyramid differs"
    assert (counts > 0).sum() > 0 and r0[..., :3].sum() > 0
    ctx.close()


@pytest.mark.parametrize("case", ["dense_voxel", "large_kd"])
def test_voxelize_packed_sums_fallback(gpu_ready, oracle_mod, case):
    """K1's packed accumulators (two 16.16 sums per 64-bit atomic) are exact while a voxel's
    count x max|value| < 2^31.  dense_voxel: 40 000 small triangles in one voxel (count
    40 000 x 65 536 > 2^31) -- the packed pass flags the overflow and K1 repeats unpacked;
    large_kd: Kd = 300 (max|value| ~ 2^24.2) -- too few hits fit, K1 goes unpacked at once.
    Sums, counts and voxels equal the oracle's either way, and a normal scene afterwards
    packs again."""
    from vct import Context
    n = 8
    rng = np.random.default_rng(11)
    T = 40000 if case == "dense_voxel" else 64
    c = np.array([4.5, 4.5, 4.5], np.float32) / n           # one voxel's centre (unit box)
    v = (c + rng.uniform(-0.3, 0.3, (T, 3, 3)).astype(np.float32) / n).reshape(-1, 3)
    if case == "large_kd":
        v = rng.uniform(0.05, 0.95, (T * 3, 3)).astype(np.float32)
    idx = np.arange(3 * T, dtype=np.uint32)
    mat = (np.arange(T) % 2).astype(np.uint32)
    kd = np.array([[0.9, 0.2, 1.0, 1.0], [0.3, 1.0, 0.1, 1.0]], np.float32)
    if case == "large_kd":
        kd = kd * 300.0
    ctx = Context(n, (0.0, 0.0, 0.0), 1.0)
    for _ in range(2):
        ctx.voxelize(v, idx, mat, kd)
        ref_s, ref_c = oracle_mod.voxelize(n, (0.0, 0.0, 0.0), 1.0, v, idx, mat, kd)
        sums, counts = ctx.download_accum()
        assert np.array_equal(counts, ref_c) and np.array_equal(sums, ref_s)
        if case == "dense_voxel":
            assert counts.max() > 32768
        ref = oracle_mod.resolve(n, ref_s, ref_c)
        ao, nm = ctx.download_voxels()
        assert np.array_equal(ao, ref[0]) and np.array_equal(nm, ref[1])
    # a normal scene after the fallback: packed again, still exact
    s, (v2, i2, m2, k2) = scene_arrays("cornell")
    from vct import scenes
    g0, E = scenes.grid_for_unit_box(n)
    ctx2 = Context(n, g0, E)
    ctx2.voxelize(v2, i2, m2, k2)
    ref_s, ref_c = oracle_mod.voxelize(n, g0, E, v2, i2, m2, k2)
    sums, counts = ctx2.download_accum()
    assert np.array_equal(counts, ref_c) and np.array_equal(sums, ref_s)
    ctx.close()
    ctx2.close()


@pytest.mark.parametrize("name,n", [("atrium", 128), ("atrium", 256), ("courtyard", 256)])
def test_inject_bitexact_coarse_bricks(gpu_ready, oracle_mod, name, n):
    """K2 where the shadow walk's coarse bricks hold 2^3 / 4^3 voxels (n = 128 / 256; the
    sizes above use one voxel per brick) and the walk skips empty ones whole (round 5):
    level 0 equals the oracle's inject of the GPU's own voxels bit for bit, for the scene
    light, lights with one and two zero components (axis-parallel walks) and the diagonal
    (equal t on all three axes at every step: the tie order decides every cell)."""
    from vct import scenes
    ctx, s, _, _ = gpu_pipeline(n, name)
    ao, nm = ctx.download_voxels()
    for light in (scenes.LIGHT_DIR, (0.0, 1.0, -0.35), (0.0, 1.0, 0.0), (1.0, 1.0, 1.0), (-0.4, 0.7, 0.3)):
        ctx.inject_directional(light, scenes.LIGHT_COLOR)
        ref = oracle_mod.inject(n, ao, nm, light, scenes.LIGHT_COLOR)
        assert np.array_equal(ctx.download_level(0), ref), f"K2 radiance differs (light {light})"
    ctx.close()


@pytest.mark.parametrize("aniso", [True, False])
@pytest.mark.parametrize("n", [4, 8, 32, 64, 128])
def test_mips_bitexact_random_level0(gpu_ready, oracle_mod, aniso, n):
    """K3 on random level 0: every size path of the launch plan (n = 4, 8: blocks smaller
    than 8 x 8 x 4 parents; 32..128: full blocks, then a short top launch), built twice --
    bit-exact vs the oracle."""
    from vct import Context
    rng = np.random.default_rng(3 + n)
    a = (rng.random((n, n, n)) < 0.3).astype(np.float32)
    r0 = np.concatenate([rng.random((n, n, n, 3)).astype(np.float32) * a[..., None], a[..., None]], -1)
    ctx = Context(n, (0, 0, 0), 1.0, aniso=aniso)
    ctx.upload_level0(r0)
    ref = oracle_mod.build_mips(n, r0, aniso)
    for _ in range(2):
        ctx.build_mips()
        assert np.array_equal(gpu_pyramid_flat(ctx), ref)
    ctx.close()


@pytest.mark.parametrize("plan", [{"VCT_K3_BZ": "8"}, {"VCT_K3_BZ": "2"}, {"VCT_K3_PLAN": "level"}],
                         ids=["block8", "block2", "per-level"])
def test_mips_alternate_plans_bitexact(gpu_ready, oracle_mod, tmp_path, plan):
    """The K3 launch plans kept for A/B (8^3 and 8x8x2 parent blocks, per-level kernels;
    chosen once per process from the environment) build the same pyramid as the oracle:
    a child process builds random level 0s at every size path, the parent compares."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cases = [(n, aniso) for n in (4, 16, 64, 128) for aniso in (True, False)]
    ins = {}
    for n, aniso in cases:
        rng = np.random.default_rng(11 + n)
        a = (rng.random((n, n, n)) < 0.3).astype(np.float32)
        ins[f"r{n}"] = np.concatenate([rng.random((n, n, n, 3)).astype(np.float32) * a[..., None], a[..., None]], -1)
    np.savez(str(tmp_path / "in.npz"), **ins)
    child = (
        "import sys, numpy as np\n"
        f"sys.path[:0] = [{repo!r}, {os.path.join(repo, 'tests')!r}, "
        f"{os.path.join(repo, 'voxel-based-global-illumination_amd')!r}]\n"
        "from vct import Context\n"
        "from helpers import gpu_pyramid_flat\n"
        f"d = np.load({str(tmp_path / 'in.npz')!r}); out = {{}}\n"
        f"for n, aniso in {cases!r}:\n"
        "    c = Context(n, (0, 0, 0), 1.0, aniso=aniso); c.upload_level0(d[f'r{n}'])\n"
        "    c.build_mips(); out[f'p{n}_{int(aniso)}'] = gpu_pyramid_flat(c); c.close()\n"
        f"np.savez({str(tmp_path / 'out.npz')!r}, **out)\n")
    p = subprocess.run([sys.executable, "-c", child], env={**os.environ, **plan}, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    out = np.load(str(tmp_path / "out.npz"))
    for n, aniso in cases:
        assert np.array_equal(out[f"p{n}_{int(aniso)}"], oracle_mod.build_mips(n, ins[f"r{n}"], aniso)), (n, aniso)


def test_mips_constant_kat_gpu(gpu_ready):
    """KAT 2 on the GPU: constant (L*alpha, alpha) -> a_l = 1 - (1-alpha)^(2^l)."""
    from vct import Context
    n, alpha, Lr = 16, 0.3, 0.8
    r0 = np.empty((n, n, n, 4), np.float32)
    r0[..., :3] = Lr * alpha
    r0[..., 3] = alpha
    ctx = Context(n, (0, 0, 0), 1.0, aniso=True)
    ctx.upload_level0(r0)
    ctx.build_mips()
    for l in range(1, ctx.num_levels):
        al = 1 - (1 - alpha) ** (2 ** l)
        for f in range(6):
            t = ctx.download_level(l, f)
            np.testing.assert_allclose(t[..., 3], al, rtol=2e-6)
            np.testing.assert_allclose(t[..., :3], Lr * al, rtol=2e-6)
    ctx.close()


def _gbuf(kind, s, ctx_or_ref, g0, E, w, h):
    """G-buffers that drive each K4 brick mode: "scene" (flat surfaces: combined
    faces, brick cache), "rand" (per-lane gathers), "mirror" (lanes with normals
    +-n_x: equal d^2, different faces), "jitter" (one axis of the normal near
    zero with random sign: four-face bricks)."""
    from vct import scenes
    from vct.camera import Camera
    cam = Camera()
    if kind == "scene":
        return scenes.raycast_numpy(s, cam, w, h), cam
    if kind in ("mirror", "jitter"):
        pos, nrm, alb = scenes.raycast_numpy(s, cam, w, h)
        yy, xx = np.mgrid[0:h, 0:w]
        if kind == "mirror":
            sgn = np.where((xx + yy) % 2 == 0, 1.0, -1.0)
            nv = np.stack([0.6 * sgn, np.full_like(sgn, 0.8), np.zeros_like(sgn)], -1)
        else:
            rng = np.random.default_rng(5)
            nv = np.stack([rng.uniform(-0.05, 0.05, (h, w)), np.full((h, w), 0.9), np.full((h, w), 0.4)], -1)
            nv /= np.linalg.norm(nv, axis=-1, keepdims=True)
        nrm = nrm.copy()
        nrm[..., :3] = np.where(pos[..., 3:4] != 0, nv, nrm[..., :3]).astype(np.float32)
        return (pos, nrm, alb), cam
    ao, nm = ctx_or_ref
    return scenes.gbuffer_rand(ao, nm, g0, E, w, h, seed=42), cam


@pytest.mark.parametrize("name,n,kind,aniso,nd,spec", [
    ("cornell", 32, "scene", True, 9, True),
    ("cornell", 32, "rand", True, 9, True),
    ("atrium", 64, "scene", True, 9, True),
    ("atrium", 32, "rand", False, 9, True),
    ("cornell", 16, "scene", True, 1, False),
    ("atrium", 32, "rand", True, 16, True),
    ("cornell", 64, "scene", True, 0, True),
])
def test_trace_parity(gpu_ready, oracle_mod, name, n, kind, aniso, nd, spec):
    O = oracle_mod
    ctx, s, (v, i, m, k), (g0, E) = gpu_pipeline(n, name, aniso=aniso, n_diffuse=nd, specular=spec)
    (pos, nrm, alb), cam = _gbuf(kind, s, ctx.download_voxels(), g0, E, 64, 48)
    got = ctx.trace(pos, nrm, alb, cam.position)
    r0 = ctx.download_level(0)
    ref = O.trace(n, g0, E, r0, gpu_pyramid_flat(ctx), pos, nrm, alb, cam.position, aniso=aniso,
                  n_diffuse=nd, specular=spec)
    e_d = rel_l2(got["diffuse"], ref["diffuse"])
    e_s = rel_l2(got["spec"], ref["spec"]) if spec else 0.0
    both = rel_l2(np.concatenate([got["diffuse"], got["spec"]]), np.concatenate([ref["diffuse"], ref["spec"]]))
    assert both <= TRACE_TOL, (e_d, e_s)
    assert got["cone_steps"] == ref["cone_steps"]
    assert np.array_equal(got["steps_px"], ref["steps_px"])
    # the spec's operation order is shared, so the result is expected bit-exact
    assert np.array_equal(got["diffuse"], ref["diffuse"]) and np.array_equal(got["spec"], ref["spec"])
    ctx.close()


@pytest.mark.parametrize("n", [16, 64, 128])
def test_mips_relight_sparse_bitexact(gpu_ready, oracle_mod, n):
    """Relight builds (Grid::k3_live): after K2 level 0 is nonzero exactly at the occupied
    voxels, so a build that follows another from the same occupancy skips K3's blocks
    without an occupied voxel and the K4 maps.  A light sequence, a scene change (K1 ->
    full build), a dense upload in between (full build) and back: every pyramid equals
    the oracle's, and frames traced after a skipping build equal a fresh context's."""
    from vct import Context, scenes
    from helpers import scene_arrays
    g0, E = scenes.grid_for_unit_box(n)
    lights = [scenes.LIGHT_DIR, (0.3, 0.9, -0.2), (-0.5, 0.4, 0.6)]
    w, h = 64, 48
    rng = np.random.default_rng(5 + n)
    pos = np.zeros((h, w, 4), np.float32)
    pos[..., :3] = np.array(g0, np.float32) + rng.uniform(0.1, 0.9, (h, w, 3)).astype(np.float32) * E
    pos[..., 3] = 1.0
    nv = rng.standard_normal((h, w, 3))
    nrm = np.zeros((h, w, 4), np.float32)
    nrm[..., :3] = nv / np.linalg.norm(nv, axis=-1, keepdims=True)
    alb = np.full((h, w, 4), 0.5, np.float32)
    eye = (0.0, 0.5, 3.0)
    ctx = Context(n, g0, E)

    def check(name, light, arrays):
        v, i, m, k = arrays
        ref = oracle_mod.pipeline(n, g0, E, v, i, m, k, light)
        assert np.array_equal(ctx.download_level(0), ref["r0"]), (name, light)
        assert np.array_equal(gpu_pyramid_flat(ctx), ref["pyr"]), (name, light)
        fresh = Context(n, g0, E)
        fresh.voxelize(v, i, m, k)
        fresh.inject_directional(light, scenes.LIGHT_COLOR)
        fresh.build_mips()
        a, b = ctx.trace(pos, nrm, alb, eye), fresh.trace(pos, nrm, alb, eye)
        for key in ("diffuse", "spec", "steps_px"):
            assert np.array_equal(a[key], b[key]), (name, light, key)
        fresh.close()

    for name in ("atrium", "cornell"):
        _, arrays = scene_arrays(name)
        ctx.voxelize(*arrays)
        for light in lights:                     # the first build is full, the others skip
            ctx.inject_directional(light, scenes.LIGHT_COLOR)
            ctx.build_mips()
            check(name, light, arrays)
    # a dense level 0 (no K2): a full build from it, then K2 again
    ctx.upload_level0(rng.random((n, n, n, 4)).astype(np.float32) * (rng.random((n, n, n, 1)) < 0.1))
    ctx.build_mips()
    assert np.array_equal(gpu_pyramid_flat(ctx), oracle_mod.build_mips(n, ctx.download_level(0), True))
    for light in lights[:2]:
        ctx.inject_directional(light, scenes.LIGHT_COLOR)
        ctx.build_mips()
        check("cornell", light, arrays)
    ctx.close()


@pytest.mark.parametrize("n", [16, 64])
def test_empty_space_maps_exact(gpu_ready, oracle_mod, n, monkeypatch):
    """K4's empty-space test (Grid::zmap, rebuilt by build_mips from the level-0 texels
    K3 reads): a sparse uploaded level 0 with signed values, -0.0, denormals and alpha-0
    texels, traced from random surface points and normals with random roughness.  The
    frame equals the oracle bit for bit, and equals the frame traced without the maps
    (VCT_ZMAP=0); steps and per-pixel steps too."""
    from vct import Context
    rng = np.random.default_rng(17 + n)
    occ = rng.random((n, n, n)) < 0.02
    r0 = np.zeros((n, n, n, 4), np.float32)
    r0[occ] = rng.standard_normal((int(occ.sum()), 4)).astype(np.float32)
    free = np.argwhere(~occ)
    pick = free[rng.choice(len(free), 60, replace=False)]
    r0[tuple(pick[:20].T)] = -0.0                                   # negative zero: not +0
    r0[tuple(pick[20:40].T)] = np.float32(1e-40)                    # denormal
    r0[tuple(pick[40:].T)] = np.array([0.5, -0.25, 0.125, 0.0], np.float32)   # colour with alpha 0
    w, h = 96, 64
    pos = np.zeros((h, w, 4), np.float32)
    pos[..., :3] = rng.uniform(0.05, 0.95, (h, w, 3))
    pos[..., 3] = (rng.random((h, w)) < 0.9).astype(np.float32)
    nv = rng.standard_normal((h, w, 3))
    nrm = np.zeros((h, w, 4), np.float32)
    nrm[..., :3] = nv / np.linalg.norm(nv, axis=-1, keepdims=True)
    alb = np.zeros((h, w, 4), np.float32)
    alb[..., :3] = rng.random((h, w, 3))
    alb[..., 3] = rng.uniform(0.0, 1.0, (h, w))
    eye = (0.5, 0.6, 2.5)
    ctx = Context(n, (0, 0, 0), 1.0)
    ctx.upload_level0(r0)
    ctx.build_mips()
    got = ctx.trace(pos, nrm, alb, eye)
    ref = oracle_mod.trace(n, (0, 0, 0), 1.0, r0, gpu_pyramid_flat(ctx), pos, nrm, alb, eye)
    for key in ("diffuse", "spec", "steps_px"):
        assert np.array_equal(got[key], ref[key]), key
    monkeypatch.setenv("VCT_ZMAP", "0")
    ctx.build_mips()
    off = ctx.trace(pos, nrm, alb, eye)
    for key in ("diffuse", "spec", "steps_px"):
        assert np.array_equal(got[key], off[key]), key
    ctx.close()


@pytest.mark.parametrize("kind", ["scene", "jitter"])
def test_occupancy_form_curved_bitexact(gpu_ready, oracle_mod, kind):
    """Curved surfaces in the occupancy form: cones whose valid lanes select four faces
    stage 4 x 4 x 3 bricks (four 54-slot face blocks) instead of gathering per lane;
    the courtyard's columns and the jittered normals make many such waves.  Forced
    occupancy form, screen order and reordered, with and without counters: bit-exact."""
    import torch
    from vct import scenes
    from vct.camera import Camera
    n, w, h = 64, 192, 128
    ctx, s, arrs, (g0, E) = gpu_pipeline(n, "courtyard")
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    cam = Camera()
    gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)       # the raster (1 M triangles)
    torch.cuda.synchronize()
    pos, nrm, alb = (g.cpu().numpy() for g in gb)
    assert (pos[..., 3] != 0).mean() > 0.5
    if kind == "jitter":
        rng = np.random.default_rng(9)
        nv = np.stack([rng.uniform(-0.05, 0.05, (h, w)), np.full((h, w), 0.9), np.full((h, w), 0.4)], -1)
        nv /= np.linalg.norm(nv, axis=-1, keepdims=True)
        nrm = nrm.copy()
        nrm[..., :3] = np.where(pos[..., 3:4] != 0, nv, nrm[..., :3]).astype(np.float32)
        gb[1] = torch.from_numpy(nrm).to(dev)
    ref = oracle_mod.trace(n, g0, E, ctx.download_level(0), gpu_pyramid_flat(ctx), pos, nrm, alb, cam.position)
    for variant, counted in ((0x6000000, True), (0x2008000, True), (0x6000000, False), (0x2008000, False)):
        d = torch.full((h, w, 4), -1.0, device=dev)
        sp = torch.full((h, w, 4), -1.0, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.trace_device(*gb, w, h, cam.position, d, sp, cone_steps=cnt if counted else None, variant=variant)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), ref["diffuse"]), f"variant {variant:#x} diffuse"
        assert np.array_equal(sp.cpu().numpy(), ref["spec"]), f"variant {variant:#x} spec"
        if counted:
            assert int(cnt[0]) == ref["cone_steps"]
    ctx.close()


@pytest.mark.parametrize("kind", ["scene", "rand", "mirror", "jitter"])
def test_trace_variants_bitexact(gpu_ready, oracle_mod, kind):
    """The K4 variants (0 = LDS bricks, 1 = per-lane gathers; bit 0x100 = no specular step tables,
    0x200 = all cones in one workgroup, 0x400 / 0x800 = cones split over three /
    two workgroups) equal the oracle bit for bit.  Without per-pixel step counts
    the default splits the cones over workgroups (three parts for small launches,
    with a hand-over of the diffuse sum through global scratch); those forms are
    checked as well, twice in a row (the hand-over flags reset themselves)."""
    import torch
    O = oracle_mod
    n, w, h = 64, 160, 96
    ctx, s, arrs, (g0, E) = gpu_pipeline(n, "atrium")
    (pos, nrm, alb), cam = _gbuf(kind, s, ctx.download_voxels(), g0, E, w, h)
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    gb = [torch.from_numpy(a).to(dev) for a in (pos, nrm, alb)]
    ref = O.trace(n, g0, E, ctx.download_level(0), gpu_pyramid_flat(ctx), pos, nrm, alb, cam.position)
    # 0x8000: rays reordered by the Morton code of their origin voxel (alone, with gathers)
    # 0x1000000 / 0x2000000: the union / occupancy form of the default variant
    for variant in (0, 1, 0x8000, 0x8001, 0x1000000, 0x2000000, 0x2008000, 0x4000000, 0x5000000):
        d = torch.empty((h, w, 4), device=dev)
        sp = torch.empty((h, w, 4), device=dev)
        st = torch.zeros((h, w), dtype=torch.int32, device=dev)
        cnt = torch.zeros(2, dtype=torch.int64, device=dev)
        ctx.trace_device(*gb, w, h, cam.position, d, sp, steps_px=st, cone_steps=cnt[0:1],
                         texel_fetches=cnt[1:2], variant=variant)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), ref["diffuse"]), f"variant {variant} diffuse"
        assert np.array_equal(sp.cpu().numpy(), ref["spec"]), f"variant {variant} spec"
        assert np.array_equal(st.cpu().numpy().astype(np.uint32), ref["steps_px"])
        assert int(cnt[0]) == ref["cone_steps"]
        assert int(cnt[1]) > 24 * int(cnt[0]) // 2   # >= 1 aniso level per step on average
    # bits 20-23: diffuse parts of the split (3, 4 -> 3 parts of 3 cones, 5, 9 -> one cone each)
    for variant in (0, 1, 0x100, 0x200, 0x400, 0x800, 0x400, 0x300400, 0x400400, 0x500400, 0x900400, 0x900400,
                    0x500400, 0, 0x8000, 0x8400, 0x8800, 0x8200, 0x8000, 0x1000000, 0x2000000, 0x2000400,
                    0x2000800, 0x2008000, 0x4000000, 0x6000000, 0x2400, 0x902400, 0x502400, 0x2002400, 0):
        d = torch.full((h, w, 4), -1.0, device=dev)
        sp = torch.full((h, w, 4), -1.0, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.trace_device(*gb, w, h, cam.position, d, sp, cone_steps=cnt, variant=variant)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), ref["diffuse"]), f"variant {variant:#x} diffuse (no steps_px)"
        assert np.array_equal(sp.cpu().numpy(), ref["spec"]), f"variant {variant:#x} spec (no steps_px)"
        assert int(cnt[0]) == ref["cone_steps"]
    # no counters at all: the form compiled without the counting instructions (the
    # bench's timed launches), and 0x4000 = the counting form without counters
    for variant in (0, 0x4000, 0x400, 0x800, 0x200, 0x500400, 0x300400, 0x902400, 0):
        d = torch.full((h, w, 4), -1.0, device=dev)
        sp = torch.full((h, w, 4), -1.0, device=dev)
        ctx.trace_device(*gb, w, h, cam.position, d, sp, variant=variant)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), ref["diffuse"]), f"variant {variant:#x} diffuse (no counters)"
        assert np.array_equal(sp.cpu().numpy(), ref["spec"]), f"variant {variant:#x} spec (no counters)"
    # variants retired in round 4 (vct_variants.h) are refused, not silently remapped
    from vct import VctError
    for variant in (2, 3, 0x1000, 0x8002):
        with pytest.raises(VctError):
            ctx.trace_device(*gb, w, h, cam.position, d, sp, variant=variant)
    ctx.close()


def test_trace_edge_cases(gpu_ready, oracle_mod):
    """1x1 frame, all-background frame, odd sizes not multiple of 64, empty grid."""
    from vct import Context
    ctx, s, arrs, (g0, E) = gpu_pipeline(16, "cornell")
    for (w, h) in [(1, 1), (65, 3), (3, 130)]:
        pos = np.zeros((h, w, 4), np.float32)
        out = ctx.trace(pos, pos, pos, (0, 0, 3))
        assert out["cone_steps"] == 0 and not out["diffuse"].any() and not out["spec"].any()
    ctx.close()
    # empty grid: diffuse = 0, AO = 1, spec = 0
    n = 16
    c2 = Context(n, g0, E)
    c2.upload_level0(np.zeros((n, n, n, 4), np.float32))
    c2.build_mips()
    rng = np.random.default_rng(0)
    pos = np.zeros((5, 7, 4), np.float32)
    pos[..., :3] = rng.uniform(-0.5, 0.5, (5, 7, 3))
    pos[..., 3] = 1
    nrm = np.zeros_like(pos)
    nrm[..., 1] = 1
    alb = np.full_like(pos, 0.1)
    out = c2.trace(pos, nrm, alb, (0, 0, 3))
    assert not out["diffuse"][..., :3].any() and np.all(out["diffuse"][..., 3] == 1) and not out["spec"].any()
    ref = oracle_mod.trace(n, g0, E, np.zeros((n, n, n, 4), np.float32), gpu_pyramid_flat(c2), pos, nrm, alb,
                           (0, 0, 3))
    assert np.array_equal(out["steps_px"], ref["steps_px"])
    c2.close()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tiled_trace_equals_full_frame(gpu_ready, world):
    """Multi-GPU tile partition on one device: every rank's compact tiles, gathered and
    un-permuted on the device, reproduce the single-rank frame bit for bit."""
    import torch
    from vct import scenes
    from vct.camera import Camera
    from vct.multi import tiles_for_rank
    ctx, s, arrs, (g0, E) = gpu_pipeline(32, "atrium")
    w, h = 200, 130
    cam = Camera()
    dev = torch.device("cuda")
    pos, nrm, alb = (torch.empty((h, w, 4), device=dev) for _ in range(3))
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.gbuffer_raycast_device(cam, w, h, scenes.ROUGHNESS, pos, nrm, alb)
    full_d = torch.empty((h, w, 4), device=dev)
    full_s = torch.empty((h, w, 4), device=dev)
    ctx.trace_device(pos, nrm, alb, w, h, cam.position, full_d, full_s)
    maxt = tiles_for_rank(w, h, 0, world)
    g_d = torch.zeros((world, maxt * 4096, 4), device=dev)
    g_s = torch.zeros((world, maxt * 4096, 4), device=dev)
    for r in range(world):
        ctx.trace_device(pos, nrm, alb, w, h, cam.position, g_d[r], g_s[r], tile_rank=r, tile_world=world,
                         tile_compact=True)
    fd = torch.empty((h, w, 4), device=dev)
    fs = torch.empty((h, w, 4), device=dev)
    ctx.untile_device(g_d, w, h, world, fd)
    ctx.untile_device(g_s, w, h, world, fs)
    torch.cuda.synchronize()
    assert torch.equal(fd, full_d) and torch.equal(fs, full_s)
    # two planes in one launch from the [world][2][max_tiles*64*64][4] layout
    both = torch.stack([g_d, g_s], 1).contiguous()
    fd2, fs2 = torch.zeros_like(fd), torch.zeros_like(fs)
    ctx.untile_planes_device(both, w, h, world, (fd2, fs2))
    torch.cuda.synchronize()
    assert torch.equal(fd2, full_d) and torch.equal(fs2, full_s)
    # host mirror of the permutation agrees with the device one
    from vct.multi import tile_offset, untile
    host = untile(g_d.cpu().numpy(), w, h, world)
    assert np.array_equal(host, full_d.cpu().numpy())
    # packed layout (gather to the presenting rank): rank r's [2][tiles(r)] tiles at
    # tile offset 2 * tile_offset(r), no padding, traced straight into its slice
    T = tiles_for_rank(w, h, 0, 1)
    packed = torch.zeros((2 * T * 4096, 4), device=dev)
    for r in range(world):
        nt, off = tiles_for_rank(w, h, r, world), 2 * tile_offset(w, h, r, world) * 4096
        if nt:
            sl = packed[off:off + 2 * nt * 4096].view(2, nt * 4096, 4)
            ctx.trace_device(pos, nrm, alb, w, h, cam.position, sl[0], sl[1], tile_rank=r, tile_world=world,
                             tile_compact=True)
    fd3, fs3 = torch.zeros_like(fd), torch.zeros_like(fs)
    ctx.untile_planes_device(packed, w, h, world, (fd3, fs3), packed=True)
    torch.cuda.synchronize()
    assert torch.equal(fd3, full_d) and torch.equal(fs3, full_s)
    ctx.close()


def test_comm_one_rank_rccl(gpu_ready):
    """vct_comm_* through the HIP library over a one-rank RCCL communicator (the
    one-GPU box cannot hold two RCCL ranks): broadcast of level 0 and the frame
    assembled on the root (send/recv form) and on every rank (all-gather form)
    equal the plain trace bit for bit."""
    import torch
    from vct import VCT_ALL_RANKS, Context, scenes
    from vct.camera import Camera
    ctx, s, arrs, (g0, E) = gpu_pipeline(32, "atrium")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.comm_init(Context.comm_get_id(), 1, 0)
    ctx.comm_broadcast_level0(0)
    ctx.build_mips()
    w, h = 200, 130
    cam = Camera()
    dev = torch.device("cuda")
    pos, nrm, alb = (torch.empty((h, w, 4), device=dev) for _ in range(3))
    ctx.gbuffer_raycast_device(cam, w, h, scenes.ROUGHNESS, pos, nrm, alb)
    full_d, full_s = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
    ctx.trace_device(pos, nrm, alb, w, h, cam.position, full_d, full_s)
    for root in (0, VCT_ALL_RANKS):
        d, sp = torch.zeros_like(full_d), torch.zeros_like(full_s)
        ctx.comm_trace_frame(pos, nrm, alb, w, h, cam.position, d, sp, root=root)
        torch.cuda.synchronize()
        assert torch.equal(d, full_d) and torch.equal(sp, full_s), root
    # frames on alternating streams share the gather buffer (ordered on the device by
    # xchg_enter); comm_synchronize waits for the last exchange of either stream
    eyes = [(0.0, 0.0, 3.0), (0.2, 0.1, 2.6), (-0.3, 0.2, 2.8)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    outs = []
    for f, e in enumerate(eyes):
        ctx.set_stream(streams[f % 2].cuda_stream)
        d, sp = torch.empty_like(full_d), torch.empty_like(full_s)
        ctx.comm_trace_frame(pos, nrm, alb, w, h, e, d, sp, root=VCT_ALL_RANKS if f % 2 else 0)
        outs.append((d, sp))
    ctx.comm_synchronize()
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    for e, (d, sp) in zip(eyes, outs):
        ctx.trace_device(pos, nrm, alb, w, h, e, full_d, full_s)
        torch.cuda.synchronize()
        assert torch.equal(d, full_d) and torch.equal(sp, full_s), e
    ctx.comm_destroy()
    ctx.close()


def test_partial_grid_refused_gpu(gpu_ready):
    """After a voxelization with out-of-range indices the grid is partial: inject is
    refused with VCT_ESTATE until a good voxelization."""
    from vct import Context, VctError
    ctx = Context(16, (0, 0, 0), 1.0)
    v = np.zeros((3, 14), np.float32)
    ctx.voxelize(v, np.array([0, 1, 2], np.uint32))
    with pytest.raises(VctError, match="EINVAL"):
        ctx.voxelize(v, np.array([0, 1, 5], np.uint32))
    with pytest.raises(VctError, match="ESTATE"):
        ctx.inject_directional((0, 1, 0))
    ctx.voxelize(v, np.array([0, 1, 2], np.uint32))
    ctx.inject_directional((0, 1, 0))
    ctx.close()


class _FakeWork:
    def __init__(self, fn):
        self.fn = fn

    def wait(self):
        self.fn()


class _FakeGroup:
    """Stands in for an RCCL group of `world` ranks driven from ONE process: a
    rank's all_gather_into_tensor is completed when its work is waited on, from
    every rank's input of the same round (the inputs must still be intact then,
    which is exactly what FrameTracer's double buffering promises).  As with RCCL,
    an op is ordered after the work queued on the stream current when it is
    issued (an event recorded there), and a waited work orders the waiting
    stream after the copy."""

    def __init__(self, world):
        self.world, self.inputs, self.round = world, {}, [0] * world
        self.sends, self.p2p_round = {}, {}

    @staticmethod
    def _issued():
        import torch
        ev = torch.cuda.Event()
        ev.record()
        return ev

    @staticmethod
    def _after(evs):
        import torch
        for ev in evs:
            torch.cuda.current_stream().wait_event(ev)

    def view(self, rank):
        g = self

        class View:
            def get_backend(self):
                return "nccl"

            def all_gather_into_tensor(self, out, inp, async_op=False):
                rd = g.round[rank]
                g.round[rank] += 1
                g.inputs[(rd, rank)] = (inp, g._issued())

                def done():
                    g._after([g.inputs[(rd, r)][1] for r in range(g.world)])
                    for r in range(g.world):
                        out[r].copy_(g.inputs[(rd, r)][0])
                if not async_op:
                    done()
                    return None
                return _FakeWork(done)

            # point-to-point (the "present" exchange): a send is kept by reference and
            # copied when the matching receive's work is waited on (same round per pair)
            isend, irecv = "isend", "irecv"

            class P2POp:
                def __init__(self, op, tensor, peer):
                    self.op, self.tensor, self.peer = op, tensor, peer

            def batch_isend_irecv(self, ops):
                works = []
                for o in ops:
                    src, dst = (rank, o.peer) if o.op == "isend" else (o.peer, rank)
                    rd = g.p2p_round.get((src, dst, o.op), 0)
                    g.p2p_round[(src, dst, o.op)] = rd + 1
                    if o.op == "isend":
                        g.sends[(rd, src, dst)] = (o.tensor, g._issued())
                        works.append(_FakeWork(lambda: None))
                    else:
                        def recv(t=o.tensor, k=(rd, src, dst)):
                            g._after([g.sends[k][1]])
                            t.copy_(g.sends[k][0].view_as(t))
                        works.append(_FakeWork(recv))
                return works
        return View()


# overlap=None (tuned on the first step) only with one rank: the one-process fake group
# cannot run one rank's tuning frames ahead of the others
@pytest.mark.parametrize("world,mode,overlap", [(w, m, o) for w, m in ((1, "present"), (2, "present"), (3, "present"),
                                                                     (2, "allgather"), (3, "allgather"))
                                                for o in (True, False)] + [(1, "present", None)])
def test_frame_pipeline_equals_full_frames(gpu_ready, world, mode, overlap):
    """FrameTracer (bench.py's per-rank driver): the pipelined step()/drain() loop
    (the exchange of frame f overlapping the trace of frame f+1, two buffer sets,
    [diffuse | specular] moved together, one two-plane untile) yields every frame
    bit-identical to a single-rank trace of it, on rank 0 only ("present": send /
    recv of each rank's own tiles, packed) or on every rank ("allgather").  Ranks
    are FrameTracers in one process over a fake group; each frame uses a different
    eye (specular changes).  overlap: frames traced on two streams (consecutive K4
    launches run concurrently, each with its own hand-over / reorder scratch); None: the
    tracer times both on its first step (FrameTracer.tune, every rank) and keeps one."""
    import torch
    from vct import scenes
    from vct.camera import Camera
    from vct.multi import FrameTracer
    ctx, s, arrs, (g0, E) = gpu_pipeline(32, "atrium")
    w, h = 200, 130
    cam = Camera()
    dev = torch.device("cuda")
    pos, nrm, alb = (torch.empty((h, w, 4), device=dev) for _ in range(3))
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.gbuffer_raycast_device(cam, w, h, scenes.ROUGHNESS, pos, nrm, alb)
    eyes = [[float(cam.position[0]) + 0.05 * f, float(cam.position[1]), float(cam.position[2])] for f in range(4)]
    refs = []
    for e in eyes:
        d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
        ctx.trace_device(pos, nrm, alb, w, h, e, d, sp)
        refs.append((d, sp))
    grp = _FakeGroup(world)
    tr = [FrameTracer(ctx, torch, grp.view(r), w, h, r, world, dev, mode=mode, overlap=overlap)
          for r in range(world)]
    for f, e in enumerate(eyes):
        for t in tr:
            t.step((pos, nrm, alb), e)
        # one rank without overlap: the frame is done; else frame f-1 was completed inside step(f)
        # (overlap=None: the first step tuned, the tracer now runs what it chose)
        done = f if (world == 1 and not tr[0].overlap) else f - 1
        if done >= 0:
            torch.cuda.synchronize()
            for t in tr:
                if t.holds_frame:
                    assert torch.equal(t.diff, refs[done][0]) and torch.equal(t.spec, refs[done][1]), (f, t.rank)
    for t in tr:
        t.drain()
    torch.cuda.synchronize()
    assert sum(t.holds_frame for t in tr) == (1 if mode == "present" else world)
    for t in tr:
        if t.holds_frame:
            assert torch.equal(t.diff, refs[-1][0]) and torch.equal(t.spec, refs[-1][1])
    ctx.close()


def test_frame_tracer_tune(gpu_ready):
    """FrameTracer's default (overlap=None) times one stream against two on its first step
    and keeps the faster; either way the frames stay bit-identical to single traces."""
    import torch
    from vct import scenes
    from vct.camera import Camera
    from vct.multi import FrameTracer
    ctx, s, arrs, (g0, E) = gpu_pipeline(32, "atrium")
    w, h = 200, 130
    cam = Camera()
    dev = torch.device("cuda")
    gb = tuple(torch.empty((h, w, 4), device=dev) for _ in range(3))
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.gbuffer_raycast_device(cam, w, h, scenes.ROUGHNESS, *gb)
    eyes = [[float(cam.position[0]) + 0.05 * f, float(cam.position[1]), float(cam.position[2])] for f in range(3)]
    refs = []
    for e in eyes:
        d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
        ctx.trace_device(*gb, w, h, e, d, sp)
        refs.append((d, sp))
    tr = FrameTracer(ctx, torch, None, w, h, 0, 1, dev)
    assert tr.auto and tr.tuned is None
    for f, e in enumerate(eyes):
        tr.step(gb, e)
        if f == 0:
            assert not tr.auto and {"ms", "chosen", "overlap", "launch_ms", "latency_paid_ms"} == set(tr.tuned)
            assert set(tr.tuned["launch_ms"]) == set(tr.tuned["ms"])
            assert len(tr.tuned["ms"]) == 2 + tr.tune_pairs and tr.tuned["chosen"] in tr.tuned["ms"]
    tr.drain()
    torch.cuda.synchronize()
    assert torch.equal(tr.diff, refs[-1][0]) and torch.equal(tr.spec, refs[-1][1])
    ctx.close()


def test_raycast_matches_numpy(gpu_ready):
    import torch
    from vct import scenes
    from vct.camera import Camera
    ctx, s, arrs, (g0, E) = gpu_pipeline(16, "atrium")
    cam = Camera()
    w, h = 96, 64
    dev = torch.device("cuda")
    pos, nrm, alb = (torch.empty((h, w, 4), device=dev) for _ in range(3))
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.gbuffer_raycast_device(cam, w, h, 0.1, pos, nrm, alb)
    torch.cuda.synchronize()
    rp, rn, ra = scenes.raycast_numpy(s, cam, w, h, 0.1)
    gp = pos.cpu().numpy()
    valid_match = (gp[..., 3] == rp[..., 3]).mean()
    assert valid_match > 0.995
    both = (gp[..., 3] > 0) & (rp[..., 3] > 0)
    same_n = np.all(np.abs(nrm.cpu().numpy()[both] - rn[both]) < 1e-3, axis=-1).mean()
    assert same_n > 0.99
    assert np.abs(gp[both][:, :3] - rp[both][:, :3]).max() < 1e-3
    ctx.close()


@pytest.mark.parametrize("name,pos,yaw,pitch", [
    ("atrium", (0.0, 0.0, 3.0), -90.0, 0.0),       # the reference camera
    ("cornell", (0.2, -0.3, 0.5), -120.0, 20.0),   # inside the box: triangles cross the near plane
    ("random", (0.0, 0.3, 1.4), -95.0, -10.0),     # 3000-triangle soup
])
def test_raster_gbuffer_equals_raycast(gpu_ready, name, pos, yaw, pitch):
    """Row f2: the tile-binned G-buffer pass equals the brute-force ray caster bit for bit."""
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    if name == "random":
        s = scenes.random_triangles(3000, seed=9, size=0.15)
        g0, E = scenes.grid_for_unit_box(32)
        ctx = Context(32, g0, E)
        ctx.voxelize(*s.arrays())
    else:
        ctx, s, arrs, (g0, E) = gpu_pipeline(32, name)
    cam = Camera(position=pos, yaw=yaw, pitch=pitch)
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    for w, h in ((96, 64), (203, 117)):     # partial tiles on both axes
        a = [torch.full((h, w, 4), 7.0, device=dev) for _ in range(3)]
        b = [torch.full((h, w, 4), -7.0, device=dev) for _ in range(3)]
        ctx.gbuffer_raycast_device(cam, w, h, 0.1, *a)
        ctx.gbuffer_raster_device(cam, w, h, 0.1, *b)
        torch.cuda.synchronize()
        for x, y in zip(a, b):
            assert torch.equal(x, y)
        assert (a[0][..., 3] > 0).float().mean() > 0.05
    ctx.close()


def test_abi_errors(gpu_ready):
    from vct import Context, VctError
    with pytest.raises(VctError):
        Context(24, (0, 0, 0), 1.0)          # not a power of two
    with pytest.raises(VctError):
        Context(16, (0, 0, 0), -1.0)         # bad extent
    with pytest.raises(VctError):
        Context(16, (0, 0, 0), 1.0, n_diffuse=5)
    ctx = Context(16, (0, 0, 0), 1.0)
    z = np.zeros((2, 2, 4), np.float32)
    with pytest.raises(VctError, match="ESTATE"):
        ctx.trace(z, z, z, (0, 0, 0))        # trace before mips
    with pytest.raises(VctError, match="ESTATE"):
        ctx.inject_directional((0, 1, 0))    # inject before voxelize
    v = np.zeros((3, 14), np.float32)
    with pytest.raises(VctError, match="EINVAL"):
        ctx.voxelize(v, np.array([0, 1, 5], np.uint32))   # index out of range
    with pytest.raises(VctError, match="EINVAL"):
        ctx.voxelize(v, np.array([0, 1, 2], np.uint32), np.array([3], np.uint32),
                     np.ones((1, 4), np.float32))         # material out of range
    ctx.voxelize(v, np.zeros(0, np.uint32))  # empty mesh is fine
    with pytest.raises(VctError, match="EINVAL"):
        ctx.inject_directional((0, 0, 0))
    ctx.close()


def test_voxelize_reproducible_and_rerun(gpu_ready):
    """Integer atomics: reruns (and a second context) are bitwise identical."""
    ctx, s, (v, i, m, k), (g0, E) = gpu_pipeline(64, "random")
    a1 = ctx.download_accum()
    ctx.voxelize(v, i, m, k)
    a2 = ctx.download_accum()
    assert np.array_equal(a1[0], a2[0]) and np.array_equal(a1[1], a2[1])
    ctx.close()


def test_voxelize_sequence_resets_sparsely(gpu_ready, oracle_mod):
    """K1 clears only what the previous call set (records, voxels, bits): a sequence
    of different scenes on one context, and the device-resident entry point, give
    exactly the oracle's result for the last scene; K2 and the mips follow it."""
    import torch
    from vct import Context, scenes
    from helpers import scene_arrays
    n = 64
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E)
    seq = ["atrium", "cornell", "random", "atrium", "cornell"]
    for j, name in enumerate(seq):
        _, (v, i, m, k) = scene_arrays(name)
        if j % 2:
            dev = torch.device("cuda")
            ctx.voxelize_device(torch.from_numpy(v).to(dev), torch.from_numpy(i.astype(np.int32)).to(dev),
                                torch.from_numpy(m.astype(np.int32)).to(dev), torch.from_numpy(k).to(dev))
        else:
            ctx.voxelize(v, i, m, k)
        ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
        ctx.build_mips()
        ref = oracle_mod.pipeline(n, g0, E, v, i, m, k, scenes.LIGHT_DIR)
        sums, counts = ctx.download_accum()
        assert np.array_equal(counts, ref["counts"]) and np.array_equal(sums, ref["sums"]), name
        ao, nm = ctx.download_voxels()
        assert np.array_equal(ao, ref["albedo_occ"]) and np.array_equal(nm, ref["normal"]), name
        assert np.array_equal(ctx.download_level(0), ref["r0"]), name
        assert np.array_equal(gpu_pyramid_flat(ctx), ref["pyr"]), name
    # a dense level-0 upload in between: the next injection still equals the oracle's
    rng = np.random.default_rng(9)
    ctx.upload_level0(rng.random((n, n, n, 4)).astype(np.float32))
    _, (v, i, m, k) = scene_arrays("atrium")
    ctx.voxelize(v, i, m, k)
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ref = oracle_mod.pipeline(n, g0, E, v, i, m, k, scenes.LIGHT_DIR)
    assert np.array_equal(ctx.download_level(0), ref["r0"])
    # an empty mesh clears the grid
    ctx.voxelize(np.zeros((0, 14), np.float32), np.zeros(0, np.uint32))
    ao, nm = ctx.download_voxels()
    assert not ao.any() and not nm.any()
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    assert not ctx.download_level(0).any()
    ctx.close()


@pytest.mark.parametrize("name,n", [("cornell", 32), ("atrium", 64)])
def test_composite_matches_oracle(gpu_ready, oracle_mod, name, n):
    """Row f3: composite + present on the GPU equals the oracle: linear output
    bit-exact, RGBA8 within 1 (powf differs by an ulp between libm and the device)."""
    import torch
    from vct import scenes
    O = oracle_mod
    w, h = 96, 64
    ctx, s, arrs, (g0, E) = gpu_pipeline(n, name)
    (pos, nrm, alb), cam = _gbuf("scene", s, None, g0, E, w, h)
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    gb = [torch.from_numpy(a).to(dev) for a in (pos, nrm, alb)]
    d = torch.empty((h, w, 4), device=dev)
    sp = torch.empty((h, w, 4), device=dev)
    ctx.trace_device(*gb, w, h, cam.position, d, sp)
    lin = torch.empty((h, w, 4), device=dev)
    rgba = torch.empty((h, w), dtype=torch.int32, device=dev)
    ctx.composite_device(*gb, d, sp, w, h, scenes.LIGHT_DIR, scenes.LIGHT_COLOR, out_linear4=lin, out_rgba8=rgba)
    torch.cuda.synchronize()
    ao, _ = ctx.download_voxels()
    ref_lin, ref_rgba = O.composite(n, g0, E, ao, pos, nrm, alb, d.cpu().numpy(), sp.cpu().numpy(),
                                    scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    assert np.array_equal(lin.cpu().numpy(), ref_lin)
    got = rgba.cpu().numpy().view(np.uint32)
    for sh in (0, 8, 16, 24):
        a = ((got >> sh) & 255).astype(np.int64)
        b = ((ref_rgba >> sh) & 255).astype(np.int64)
        assert np.abs(a - b).max() <= 1
    assert (pos[..., 3] != 0).any() and (ref_lin[..., :3] > 0).any()
    # the shadow term matters on these scenes: some lit-facing pixels are shadowed
    ctx.close()


@pytest.mark.parametrize("name", ["atrium", "random"])
def test_backends_agree(gpu_ready, oracle_mod, name):
    """include/vct.h has two implementations, the HIP library (the
    product) and the CPU oracle backend (oracle/_build/libvct_cpu.so, test only).
    One call sequence through the same binding gives the same results from both:
    K1 sums / voxels, K2 level 0, every K3 level and face, the G-buffer of the
    ray caster and of the binned pass, the full-frame trace, a 2-rank compact
    tile split + un-permute, and the composite (linear bit-exact, RGBA8 +-1)."""
    import ctypes as C
    import torch
    from vct import Context, _lib, scenes
    from vct.camera import Camera
    cpu = _lib.bind(C.CDLL(oracle_mod.CPU_BACKEND))
    s, (v, i, m, k) = scene_arrays(name)
    n, w, h = 32, 96, 64
    g0, E = scenes.grid_for_unit_box(n)
    dev = torch.device("cuda")
    ctxs = {"hip": Context(n, g0, E), "cpu": Context(n, g0, E, lib=cpu)}
    ctxs["hip"].set_stream(torch.cuda.current_stream().cuda_stream)
    for c in ctxs.values():
        c.voxelize(v, i, m, k)
        c.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
        c.build_mips()
    a, b = ctxs["hip"], ctxs["cpu"]
    for x, y in zip(a.download_accum(), b.download_accum()):
        assert np.array_equal(x, y)
    for x, y in zip(a.download_voxels(), b.download_voxels()):
        assert np.array_equal(x, y)
    for l in range(a.num_levels):
        for f in range(a.level_dims(l)[1]):
            assert np.array_equal(a.download_level(l, f), b.download_level(l, f)), (l, f)
    cam = Camera()
    # "device" buffers: torch on the GPU, numpy for the CPU backend
    gh = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
    gc = [np.zeros((h, w, 4), np.float32) for _ in range(3)]
    for fn in ("gbuffer_raycast_device", "gbuffer_raster_device"):
        getattr(a, fn)(cam, w, h, scenes.ROUGHNESS, *gh)
        getattr(b, fn)(cam, w, h, scenes.ROUGHNESS, *[t.ctypes.data for t in gc])
        torch.cuda.synchronize()
        for x, y in zip(gh, gc):
            assert np.array_equal(x.cpu().numpy(), y), fn
    dh, sh = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
    dc, sc = np.zeros((h, w, 4), np.float32), np.zeros((h, w, 4), np.float32)
    ch, cc = torch.zeros(1, dtype=torch.int64, device=dev), np.zeros(1, np.int64)
    a.trace_device(*gh, w, h, cam.position, dh, sh, cone_steps=ch)
    b.trace_device(*[t.ctypes.data for t in gc], w, h, cam.position, dc.ctypes.data, sc.ctypes.data,
                   cone_steps=cc.ctypes.data)
    torch.cuda.synchronize()
    assert np.array_equal(dh.cpu().numpy(), dc) and np.array_equal(sh.cpu().numpy(), sc)
    assert int(ch.item()) == int(cc[0]) > 0
    from vct.multi import tiles_for_rank
    maxt = tiles_for_rank(w, h, 0, 2)
    gth = torch.zeros((2, 2, maxt * 4096, 4), device=dev)
    gtc = np.zeros((2, 2, maxt * 4096, 4), np.float32)
    for r in range(2):
        a.trace_device(*gh, w, h, cam.position, gth[r, 0], gth[r, 1], tile_rank=r, tile_world=2, tile_compact=True)
        b.trace_device(*[t.ctypes.data for t in gc], w, h, cam.position, gtc[r, 0].ctypes.data,
                       gtc[r, 1].ctypes.data, tile_rank=r, tile_world=2, tile_compact=True)
    torch.cuda.synchronize()
    assert np.array_equal(gth.cpu().numpy(), gtc)
    lin_h, rgb_h = torch.empty((h, w, 4), device=dev), torch.empty((h, w), dtype=torch.int32, device=dev)
    lin_c, rgb_c = np.zeros((h, w, 4), np.float32), np.zeros((h, w), np.uint32)
    a.composite_device(*gh, dh, sh, w, h, scenes.LIGHT_DIR, out_linear4=lin_h, out_rgba8=rgb_h)
    b.composite_device(*[t.ctypes.data for t in gc], dc.ctypes.data, sc.ctypes.data, w, h, scenes.LIGHT_DIR,
                       out_linear4=lin_c.ctypes.data, out_rgba8=rgb_c.ctypes.data)
    torch.cuda.synchronize()
    assert np.array_equal(lin_h.cpu().numpy(), lin_c)
    bh = rgb_h.cpu().numpy().view(np.uint32).view(np.uint8).astype(int)
    assert np.abs(bh - rgb_c.view(np.uint8).astype(int)).max() <= 1
    for c in ctxs.values():
        c.close()


def test_cpp_host_renderer_slot(gpu_ready, tmp_path):
    """The C++ host (host/main.cpp: the reference's Engine loop with the
    ConeTraceRenderer in its Renderer slot, OBJ loaded by the in-repo assimp-3.3
    equivalent) renders frames on the GPU through the C-ABI: every frame takes the
    same cone steps, a rerun writes the same image, and the step count matches the
    Python binding's trace of the same scene (the C++ camera derives its vectors in
    float, the Python one in double, so pixels may differ in the last bit)."""
    import os
    import re
    import subprocess
    import torch
    from helpers import write_obj
    from vct import Context, scenes
    from vct.camera import Camera
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "voxel-based-global-illumination_amd", "build", "vct_headless")
    assert os.path.exists(exe), "build the host with `make -C voxel-based-global-illumination_amd host`"
    s = scenes.atrium()
    obj = write_obj(s, str(tmp_path))
    n, w, h = 64, 160, 120
    runs = []
    for r in range(2):
        out = str(tmp_path / f"frame{r}.ppm")
        p = subprocess.run([exe, obj, str(n), str(w), str(h), "3", out, "--model=identity", "--grid=unit"],
                           capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr
        steps = [int(x) for x in re.findall(r"(\d+) cone steps", p.stdout)]
        assert len(steps) == 3 and len(set(steps)) == 1 and steps[0] > 0, p.stdout
        data = open(out, "rb").read()
        assert data.startswith(f"P6\n{w} {h}\n255\n".encode())
        img = np.frombuffer(data[len(f"P6\n{w} {h}\n255\n"):], np.uint8).reshape(h, w, 3)
        runs.append((steps[0], img))
    assert runs[0][0] == runs[1][0] and np.array_equal(runs[0][1], runs[1][1])
    # the same host driving three device ranks through vct_create_multi: the same image
    out = str(tmp_path / "frame_multi.ppm")
    p = subprocess.run([exe, obj, str(n), str(w), str(h), "2", out, "3", "--model=identity", "--grid=unit"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert [int(x) for x in re.findall(r"(\d+) cone steps", p.stdout)] == [runs[0][0]] * 2, p.stdout
    assert open(out, "rb").read() == open(str(tmp_path / "frame0.ppm"), "rb").read()
    img = runs[0][1]
    assert len(np.unique(img.reshape(-1, 3), axis=0)) > 100          # a shaded scene, not a clear
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E)
    ctx.voxelize(*s.arrays())
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ctx.build_mips()
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
    cam = Camera()
    ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)
    d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.trace_device(*gb, w, h, cam.position, d, sp, cone_steps=cnt)
    torch.cuda.synchronize()
    assert abs(int(cnt.item()) - runs[0][0]) <= 0.01 * runs[0][0], (int(cnt.item()), runs[0][0])
    ctx.close()


@pytest.mark.parametrize("devices", [1, 2, 3])
def test_multi_device_context(gpu_ready, devices):
    """vct_create_multi (one process, several GPUs): the frame split over
    `devices` ranks -- each traces its 64x64 tiles, the others' tiles reach device 0 by
    peer copies, device 0 un-permutes -- equals a single-device context bit for bit
    (outputs, per-pixel steps, counters), through the host and the device entry points,
    and after the light changes (level 0 re-sent to the other devices).  On a one-GPU
    box the ranks share the device (device r = r mod device count), which exercises the
    same copies and ordering."""
    import torch
    from vct import Context, VctError, scenes
    n, w, h = 64, 200, 136            # partial tiles at the right and bottom edges
    ref, s, (v, i, m, k), (g0, E) = gpu_pipeline(n, "atrium")
    ctx = Context(n, g0, E, devices=devices)
    assert ctx.num_devices == devices
    ctx.voxelize(v, i, m, k)
    (pos, nrm, alb), cam = _gbuf("scene", s, None, g0, E, w, h)
    dev = torch.device("cuda")
    gb = [torch.from_numpy(a).to(dev) for a in (pos, nrm, alb)]
    for light in (scenes.LIGHT_DIR, (-0.4, 1.0, 0.3)):
        for c in (ref, ctx):
            c.inject_directional(light, scenes.LIGHT_COLOR)
            c.build_mips()
        for l in range(ref.num_levels):
            for f in range(ref.level_dims(l)[1]):
                assert np.array_equal(ctx.download_level(l, f), ref.download_level(l, f)), (l, f)
        a, b = ref.trace(pos, nrm, alb, cam.position), ctx.trace(pos, nrm, alb, cam.position)
        for key in ("diffuse", "spec", "steps_px"):
            assert np.array_equal(a[key], b[key]), f"{devices} devices: {key} (host entry point)"
        assert a["cone_steps"] == b["cone_steps"]
        for counters in (True, False):
            outs = []
            for c in (ref, ctx):
                d = torch.full((h, w, 4), -1.0, device=dev)
                sp = torch.full((h, w, 4), -1.0, device=dev)
                cnt = torch.zeros(2, dtype=torch.int64, device=dev) if counters else None
                c.trace_device(*gb, w, h, cam.position, d, sp, cone_steps=cnt[0:1] if counters else None,
                               texel_fetches=cnt[1:2] if counters else None)
                c.synchronize()
                outs.append((d, sp, cnt))
            (d0, s0, c0), (d1, s1, c1) = outs
            assert torch.equal(d0, d1) and torch.equal(s0, s1), f"{devices} devices: device entry point"
            if counters:
                assert torch.equal(c0, c1), (c0.tolist(), c1.tolist())
    if devices > 1:
        d = torch.empty((h, w, 4), device=dev)
        with pytest.raises(VctError):
            ctx.trace_device(*gb, w, h, cam.position, d, d.clone(), tile_rank=0, tile_world=2)
    # frames queued on alternating streams without a host wait share the gather buffer:
    # each exchange waits on the device for the previous one (xchg_enter), so every frame
    # equals the single-device frame of its eye
    eyes = [(0.0, 0.0, 3.0), (0.2, 0.1, 2.6), (-0.3, 0.2, 2.8), (0.1, -0.2, 3.2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    got = []
    for f, e in enumerate(eyes):
        st = streams[f % 2]
        ctx.set_stream(st.cuda_stream)
        d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
        with torch.cuda.stream(st):
            ctx.trace_device(*gb, w, h, e, d, sp)
        got.append((d, sp))
    ctx.synchronize()
    torch.cuda.synchronize()
    ref.set_stream(torch.cuda.current_stream().cuda_stream)
    for e, (d, sp) in zip(eyes, got):
        rd, rs = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
        ref.trace_device(*gb, w, h, e, rd, rs)
        torch.cuda.synchronize()
        assert torch.equal(d, rd) and torch.equal(sp, rs), f"{devices} devices: frame on alternating streams, eye {e}"
    ctx.close()
    ref.close()


def test_cpp_host_reference_placement(gpu_ready, tmp_path):
    """ConeTraceRenderer with the reference's draw placement (host/main.cpp defaults):
    the model matrix T(0,-1.75,0) S(0.2) of r_voxelization.cpp:26-29 applied before
    K1 and the grid fitted around the placed model.  The host's grid equals
    vcth_grid_for_bounds of the placed bounds, and its frames take the cone steps of
    the Python path voxelizing the same placed vertices (host loader + host
    transform) in that grid (within 1 %: float vs double camera vectors)."""
    import os
    import re
    import subprocess
    import torch
    import host_lib
    from helpers import write_obj
    from vct import Context, scenes
    from vct.camera import Camera, reference_model_matrix
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "voxel-based-global-illumination_amd", "build", "vct_headless")
    s = scenes.atrium()
    s.verts = [[5.0 * r[0], 5.0 * r[1], 5.0 * r[2]] + list(r[3:]) for r in s.verts]   # nanosuit-sized: y in [-2.75, -0.75] after M
    obj = write_obj(s, str(tmp_path))
    n, w, h = 64, 160, 120
    p = subprocess.run([exe, obj, str(n), str(w), str(h), "2", str(tmp_path / "placed.ppm")], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    g = re.search(r"aabb_min (\S+) (\S+) (\S+) extent (\S+)", p.stdout)
    g0 = [float.fromhex(x) for x in g.groups()[:3]]
    E = float.fromhex(g.group(4))
    steps = [int(x) for x in re.findall(r"(\d+) cone steps", p.stdout)]
    v, i, m, k, lo, hi = host_lib.load_placed(obj, reference_model_matrix())
    assert lo[1] >= np.float32(-2.75) - 1e-5 and hi[1] <= np.float32(-0.75) + 1e-5
    hg0, hE = host_lib.grid_for_bounds(lo, hi, n)
    assert np.array_equal(np.float32(g0), hg0) and np.float32(E) == np.float32(hE)
    ctx = Context(n, g0, E)
    ctx.voxelize(v, i, m, k)
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ctx.build_mips()
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
    cam = Camera()
    ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)
    d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.trace_device(*gb, w, h, cam.position, d, sp, cone_steps=cnt)
    torch.cuda.synchronize()
    pos = gb[0].cpu().numpy()
    hit = pos[..., 3] != 0
    assert hit.sum() > 0.05 * w * h                  # the placed model is in view
    assert pos[hit][:, 1].max() <= hi[1] + 1e-4      # every hit lies on the moved geometry
    assert steps and len(set(steps)) == 1 and abs(int(cnt.item()) - steps[0]) <= 0.01 * steps[0]
    ctx.close()


@pytest.mark.parametrize("case,size", [(0, "200x130"), (1, "160x120"), (2, "64x48"), (5, "200x130")])
def test_gbuffer_projects_to_pixel_centres(gpu_ready, case, size):
    """The G-buffer pass against the reference camera: every hit position of the HIP
    raster pass, projected through GLM's perspective(radians(Zoom), w/h, 0.1, 100) and
    lookAt view matrix of the reference Camera (tests/golden/ref_camera.json, from the
    reference's own camera.cpp + GLM), lands on its pixel centre within 1e-3 px
    (row 0 = top).  The camera is the fixture's Position/Front/Up/Right/Zoom."""
    import json
    import os
    import torch
    from vct import VctCamera, scenes
    fix = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_camera.json")))
    c = fix["cameras"][case]
    hx = lambda v: np.array([float.fromhex(x) for x in v], np.float64)
    w, h = (int(x) for x in size.split("x"))
    ctx, s, arrs, (g0, E) = gpu_pipeline(32, "atrium")
    vc = VctCamera()
    vc.position[:], vc.front[:] = list(hx(c["position"])), list(hx(c["front"]))
    vc.up[:], vc.right[:] = list(hx(c["up"])), list(hx(c["right"]))
    vc.zoom_deg, vc.near_plane, vc.far_plane = float.fromhex(c["zoom"]), 0.1, 100.0
    dev = torch.device("cuda")
    gb = [torch.zeros((h, w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(vc, w, h, scenes.ROUGHNESS, *gb)
    torch.cuda.synchronize()
    pos = gb[0].cpu().numpy().astype(np.float64)
    hit = pos[..., 3] != 0
    assert hit.sum() > 0.2 * w * h
    V = hx(c["view"]).reshape(4, 4).T
    P = hx(c["proj"][size]).reshape(4, 4).T
    ys, xs = np.nonzero(hit)
    p4 = np.concatenate([pos[ys, xs, :3], np.ones((len(xs), 1))], 1)
    clip = p4 @ (P @ V).T
    ndc = clip[:, :3] / clip[:, 3:4]
    px = (ndc[:, 0] + 1.0) * 0.5 * w
    py = (1.0 - ndc[:, 1]) * 0.5 * h
    err = np.maximum(np.abs(px - (xs + 0.5)), np.abs(py - (ys + 0.5)))
    assert err.max() <= 1e-3, (err.max(), np.argmax(err))
    assert np.all((ndc[:, 2] > -1) & (ndc[:, 2] < 1))     # inside GLM's depth range (near 0.1, far 100)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["rand", "scene"])
def test_reorder_equals_screen_order(gpu_ready, kind):
    """Ray reordering (variant 0x8000) at the metric size (256^3, 1080p, 9 + 1 cones):
    the outputs, per-pixel step counts and step counter equal the screen-order trace
    bit for bit, for the incoherent G_rand it is meant for and for G_scene; the timed
    launch form (no counters) too."""
    import torch
    from vct import scenes
    n, w, h = 256, 1920, 1080
    ctx, s, arrs, (g0, E) = gpu_pipeline(n, "atrium")
    from vct.camera import Camera
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    cam = Camera()
    if kind == "scene":
        gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
        ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)
    else:
        ao, nm = ctx.download_voxels()
        gb = [torch.from_numpy(x).to(dev) for x in scenes.gbuffer_rand(ao, nm, g0, E, w, h, seed=42)]
    outs = {}
    for variant in (0, 0x8000):
        d = torch.full((h, w, 4), -1.0, device=dev)
        sp = torch.full((h, w, 4), -1.0, device=dev)
        st = torch.zeros((h, w), dtype=torch.int32, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.trace_device(*gb, w, h, cam.position, d, sp, steps_px=st, cone_steps=cnt, variant=variant)
        d2 = torch.full((h, w, 4), -1.0, device=dev)
        sp2 = torch.full((h, w, 4), -1.0, device=dev)
        ctx.trace_device(*gb, w, h, cam.position, d2, sp2, variant=variant)   # timed form
        torch.cuda.synchronize()
        outs[variant] = (d, sp, st, int(cnt[0]), d2, sp2)
    a, b = outs[0], outs[0x8000]
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), "reordered outputs differ"
    assert torch.equal(a[2], b[2]) and a[3] == b[3], "reordered step counts differ"
    assert torch.equal(b[4], a[0]) and torch.equal(b[5], a[1]), "reordered timed form differs"
    assert torch.equal(a[4], a[0]) and torch.equal(a[5], a[1])


@pytest.mark.gpu
def test_reordered_frames_overlapped(gpu_ready):
    """Consecutive ray-reordered frames (variant 0x8000: key kernel, radix sort, K4) traced
    concurrently on two streams (FrameTracer overlap): each stream has its own key / sort
    scratch, so every frame equals its single-stream trace bit for bit."""
    import torch
    from vct import scenes
    from vct.multi import FrameTracer
    n, w, h = 32, 320, 200
    ctx, s, arrs, (g0, E) = gpu_pipeline(n, "atrium")
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ao, nm = ctx.download_voxels()
    gb = tuple(torch.from_numpy(x).to(dev) for x in scenes.gbuffer_rand(ao, nm, g0, E, w, h, seed=7))
    eyes = [[0.05 * f, 0.0, 3.0] for f in range(6)]
    refs = []
    for e in eyes:
        d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
        ctx.trace_device(*gb, w, h, e, d, sp, variant=0x8000)
        refs.append((d, sp))
    tr = FrameTracer(ctx, torch, None, w, h, 0, 1, dev, overlap=True)
    for f, e in enumerate(eyes):
        tr.step(gb, e, variant=0x8000)
        if f >= 1:
            torch.cuda.synchronize()
            assert torch.equal(tr.diff, refs[f - 1][0]) and torch.equal(tr.spec, refs[f - 1][1]), f
    tr.drain()
    torch.cuda.synchronize()
    assert torch.equal(tr.diff, refs[-1][0]) and torch.equal(tr.spec, refs[-1][1])
    ctx.close()


@pytest.mark.gpu
def test_trace_form_tuner(gpu_ready):
    """The default variant times its two compiled forms on the first counter-free launches
    of a workload and keeps the faster one (vct_trace_form): every launch, whichever form
    ran it, gives the same bits as the counting form; the choice is made within a few
    dozen frames and restarts for a new workload (frame size)."""
    import torch
    from vct import scenes
    from vct.camera import Camera
    n = 128
    ctx, s, arrs, (g0, E) = gpu_pipeline(n, "atrium")
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    cam = Camera()
    for w, h in ((320, 200), (256, 128)):
        gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
        ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)
        ref_d = torch.empty((h, w, 4), device=dev)
        ref_s = torch.empty((h, w, 4), device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.trace_device(*gb, w, h, cam.position, ref_d, ref_s, cone_steps=cnt)   # counting form
        assert ctx.trace_form == -1 or w != 320
        d = torch.empty_like(ref_d)
        sp = torch.empty_like(ref_s)
        for i in range(64):
            d.fill_(-1.0)
            sp.fill_(-1.0)
            ctx.trace_device(*gb, w, h, cam.position, d, sp)
            torch.cuda.synchronize()
            assert torch.equal(d, ref_d) and torch.equal(sp, ref_s), f"launch {i} (form {ctx.trace_form})"
            if ctx.trace_form >= 0:
                break
        assert ctx.trace_form in (0, 1, 2, 3), "no candidate chosen after 64 launches"


@pytest.mark.gpu
def test_trace_form_tuner_alternating_workloads(gpu_ready):
    """A host that double-buffers its G-buffer, alternates counting and plain launches and
    two frame sizes keeps every choice (one tuner entry per workload, LRU): the form
    settles within a few dozen frames and never goes back to timing (-1) afterwards,
    and every launch still gives the counting form's bits."""
    import torch
    from vct import scenes
    from vct.camera import Camera
    ctx, s, arrs, (g0, E) = gpu_pipeline(128, "atrium")
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    cams = [Camera(), Camera(position=(0.1, 0.0, 2.6), yaw=-95.0)]
    work = []
    for w, h in ((320, 200), (256, 128)):
        for cam in cams:                                   # two G-buffers per size (double buffering)
            gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
            ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)
            ref_d, ref_s = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
            cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            ctx.trace_device(*gb, w, h, cam.position, ref_d, ref_s, cone_steps=cnt)
            work.append((w, h, cam, gb, ref_d, ref_s, cnt))
    forms = {}
    for i in range(160):
        w, h, cam, gb, ref_d, ref_s, cnt = work[i % len(work)]
        d, sp = torch.full_like(ref_d, -1.0), torch.full_like(ref_s, -1.0)
        if i % 3 == 2:                                     # a counting launch in between
            ctx.trace_device(*gb, w, h, cam.position, d, sp, cone_steps=cnt)
        else:
            ctx.trace_device(*gb, w, h, cam.position, d, sp)
        torch.cuda.synchronize()
        assert torch.equal(d, ref_d) and torch.equal(sp, ref_s), f"launch {i}"
        f = ctx.trace_form
        key = (w, h)
        if key in forms:
            assert f == forms[key], f"workload {key} went back to timing at launch {i}: {f}"
        elif f >= 0 and i >= 2 * len(work):
            forms[key] = f
    assert set(forms) == {(320, 200), (256, 128)}, forms


@pytest.mark.gpu
def test_trace_form_forced_reports_candidate(gpu_ready):
    """A variant that fixes both dimensions reports the forced candidate (not a stale one)."""
    import torch
    from vct import scenes
    from vct._lib import VctTraceArgs  # noqa: F401  (the binding's struct)
    from vct.camera import Camera
    ctx, s, arrs, (g0, E) = gpu_pipeline(64, "cornell")
    dev = torch.device("cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    cam = Camera()
    w, h = 128, 96
    gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)
    d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
    for variant, form in ((0x2000000 | 0x4000000, 1), (0x1000000 | 0x4000000, 0), (0x1000000 | 0x8000, 2)):
        ctx.trace_device(*gb, w, h, cam.position, d, sp, variant=variant)
        torch.cuda.synchronize()
        assert ctx.trace_form == form, (hex(variant), ctx.trace_form)


@pytest.mark.parametrize("world,rank,gbuf", [(1, 0, "scene"), (8, 3, "scene"), (3, 1, "scene"), (1, 0, "rand")])
def test_longest_first_dispatch_bitexact(gpu_ready, oracle_mod, world, rank, gbuf):
    """Longest-first dispatch (vct_trace.hip k4_lpt_bands / k4_lpt_order): once a workload's
    candidate is settled, every timed launch records each unit's wave duration and the next
    one deals each XCD's units longest first.  Every launch equals the counting launch bit
    for bit, and so does the oracle's frame:
    * the recording ones and the longest-first ones on one stream (the hook
      vct_debug_k4_lpt_launches shows that an order table was applied);
    * launches alternating between two streams, also with 0x10000000: these overlap
      another frame, so they keep blockIdx order (the order scratch is shared by the
      streams; the hook's count must not move);
    * the dispatch switched off (0x20000000)."""
    import torch
    from vct.multi import TILE, tiles_for_rank
    n, w, h = 64, 320, 192
    ctx, s, arrs, (g0, E) = gpu_pipeline(n, "atrium")
    (pos, nrm, alb), cam = _gbuf(gbuf, s, ctx.download_voxels(), g0, E, w, h)
    dev = torch.device("cuda")
    main = torch.cuda.current_stream()
    ctx.set_stream(main.cuda_stream)
    gb = [torch.from_numpy(a).to(dev) for a in (pos, nrm, alb)]
    opx = tiles_for_rank(w, h, rank, world) * TILE * TILE if world > 1 else w * h
    kw = dict(tile_rank=rank, tile_world=world, tile_compact=world > 1)

    def run(variant=0, counted=False, stream=None):
        d = torch.full((opx, 4), -1.0, device=dev)
        sp = torch.full((opx, 4), -1.0, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        if stream is not None:
            stream.wait_stream(main)
            ctx.set_stream(stream.cuda_stream)
        ctx.trace_device(*gb, w, h, cam.position, d, sp, cone_steps=cnt if counted else None, variant=variant, **kw)
        if stream is not None:
            ctx.set_stream(main.cuda_stream)
            main.wait_stream(stream)
        torch.cuda.synchronize()
        return d.cpu().numpy(), sp.cpu().numpy(), int(cnt[0])

    rd, rs, steps = run(counted=True)
    if world == 1:
        ref = oracle_mod.trace(n, g0, E, ctx.download_level(0), gpu_pyramid_flat(ctx), pos, nrm, alb, cam.position)
        assert np.array_equal(rd.reshape(h, w, 4), ref["diffuse"]) and np.array_equal(rs.reshape(h, w, 4), ref["spec"])
        assert steps == ref["cone_steps"]
    lpt = ctx.lib.vct_debug_k4_lpt_launches
    lpt.restype, lpt.argtypes = C.c_longlong, [C.c_void_p]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for i in range(32):   # settle the candidate, record, then longest-first launches
        d, sp, _ = run()
        assert np.array_equal(d, rd) and np.array_equal(sp, rs), i
    assert ctx.trace_form >= 0
    applied = lpt(ctx.h)
    assert applied > 0, "no launch was dispatched longest first"
    for i in range(16):   # two streams: never longest first, 0x10000000 or not
        d, sp, _ = run(variant=0x10000000 if i % 4 < 2 else 0, stream=streams[i % 2])
        assert np.array_equal(d, rd) and np.array_equal(sp, rs), ("two streams", i)
    assert lpt(ctx.h) == applied
    d, sp, _ = run(variant=0x20000000)
    assert np.array_equal(d, rd) and np.array_equal(sp, rs)
    ctx.close()
