"""Grid / G-buffer dump and load (include/vct.h vct_save_grid / vct_load_grid / vct_dump_info,
vct.dump; SURVEY.md §5 checkpoint / resume), on the CPU backend of include/vct.h
(oracle/_build/libvct_cpu.so; test infrastructure) and, marked gpu, on the HIP library.

* A dump with K1's state (VOXELS) makes a relightable context: dump -> reload (into a
  context that held another scene) -> a new light -> mips -> trace equals a fresh
  context that voxelized the scene and took that light, bit for bit (voxels, integer
  sums, level 0, pyramid, frame, composite).
* LEVEL0 (+ PYRAMID, verified on load) reproduces the dumped frame at once.
* The file format is one for both libraries: a dump from one loads into the other.
* A damaged dump or one of another grid (n, aabb_min, extent, aniso) is refused before
  anything changes (the grid placement is checked, not only n / aniso)."""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def cpu_lib(oracle_mod):
    from vct import _lib
    return _lib.bind(C.CDLL(oracle_mod.CPU_BACKEND))


LIGHT2 = (-0.5, 0.4, 0.6)


def _ctx(lib, n):
    from vct import Context, scenes
    g0, E = scenes.grid_for_unit_box(n)
    return Context(n, g0, E, lib=lib)


def _grid(lib, n=16, name="cornell", light=None):
    from helpers import scene_arrays
    from vct import scenes
    _, (v, i, m, k) = scene_arrays(name)
    ctx = _ctx(lib, n)
    ctx.voxelize(v, i, m, k)
    ctx.inject_directional(light or scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ctx.build_mips()
    return ctx


def _gbuf(n, w=24, h=16, seed=3):
    rng = np.random.default_rng(seed)
    pos = np.zeros((h, w, 4), np.float32)
    pos[..., :3] = rng.uniform(-0.8, 0.8, (h, w, 3))
    pos[..., 3] = (rng.random((h, w)) < 0.8).astype(np.float32)
    nv = rng.standard_normal((h, w, 3))
    nrm = np.zeros((h, w, 4), np.float32)
    nrm[..., :3] = nv / np.linalg.norm(nv, axis=-1, keepdims=True)
    alb = np.full((h, w, 4), 0.4, np.float32)
    return pos, nrm, alb, (0.0, 0.2, 2.5)


def _same_frames(a, b, gb):
    pos, nrm, alb, eye = gb
    f1, f2 = a.trace(pos, nrm, alb, eye), b.trace(pos, nrm, alb, eye)
    for key in ("diffuse", "spec", "steps_px"):
        assert np.array_equal(f1[key], f2[key]), key


def _same_grids(a, b):
    for x, y in zip(a.download_voxels(), b.download_voxels()):
        assert np.array_equal(x, y)
    for x, y in zip(a.download_accum(), b.download_accum()):
        assert np.array_equal(x, y)
    assert np.array_equal(a.download_level(0), b.download_level(0))
    for la, lb in zip(a.download_pyramid(), b.download_pyramid()):
        for fa, fb in zip(la, lb):
            assert np.array_equal(fa, fb)


def _relight_case(lib_a, lib_b, tmp_path, n=16, composite=None):
    """Scene dumped from lib_a (voxels + level 0 + pyramid) -> reloaded by lib_b into a
    context that voxelized another scene -> same frame; relit -> equal to a fresh one."""
    from helpers import scene_arrays
    from vct import dump, scenes
    a = _grid(lib_a, n, "atrium")
    dump.save_grid(a, tmp_path / "g", pyramid=True)
    info, what = dump.dump_info(tmp_path / "g", lib=lib_b)
    assert what == dump.VOXELS | dump.LEVEL0 | dump.PYRAMID and info["n"] == n
    b = _grid(lib_b, n, "cornell")                          # other scene first: the reset matters
    dump.load_grid(tmp_path / "g", ctx=b)
    gb = _gbuf(n)
    if lib_a is lib_b:
        _same_grids(a, b)
    _same_frames(a, b, gb)
    b.inject_directional(LIGHT2, scenes.LIGHT_COLOR)        # relight without the triangles
    b.build_mips()
    _, (v, i, m, k) = scene_arrays("atrium")
    c = _ctx(lib_b, n)
    c.voxelize(v, i, m, k)
    c.inject_directional(LIGHT2, scenes.LIGHT_COLOR)
    c.build_mips()
    _same_grids(b, c)
    _same_frames(b, c, gb)
    if composite:
        composite(b, c, gb)
    for x in (a, b, c):
        x.close()


def test_grid_dump_relight_cpu(cpu_lib, tmp_path):
    def composite(b, c, gb):
        pos, nrm, alb, eye = gb
        h, w = pos.shape[:2]
        outs = []
        for ctx in (b, c):
            f = ctx.trace(pos, nrm, alb, eye)
            lin = np.zeros((h, w, 4), np.float32)
            rgba = np.zeros((h, w), np.uint32)
            ctx.composite_device(pos.ctypes.data, nrm.ctypes.data, alb.ctypes.data, f["diffuse"].ctypes.data,
                                 f["spec"].ctypes.data, w, h, LIGHT2, out_linear4=lin.ctypes.data,
                                 out_rgba8=rgba.ctypes.data)
            outs.append((lin, rgba))
        assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    _relight_case(cpu_lib, cpu_lib, tmp_path, composite=composite)


@pytest.mark.parametrize("pyramid", [False, True])
def test_grid_dump_roundtrip_cpu(cpu_lib, tmp_path, pyramid):
    from vct import dump
    ctx = _grid(cpu_lib)
    dump.save_grid(ctx, tmp_path / "g", pyramid=pyramid)
    back = dump.load_grid(tmp_path / "g", lib=cpu_lib)
    assert (back.n, back.aniso) == (ctx.n, ctx.aniso)
    f32 = lambda x: np.asarray(x, np.float32)   # noqa: E731 -- the config crosses the ABI as float32
    assert np.array_equal(f32(back.extent), f32(ctx.extent)) and np.array_equal(f32(back.aabb_min), f32(ctx.aabb_min))
    _same_grids(ctx, back)
    pos, nrm, alb, eye = _gbuf(ctx.n)
    dump.save_gbuffer(tmp_path / "gb", pos, nrm, alb, eye)
    p2, n2, a2, e2 = dump.load_gbuffer(tmp_path / "gb.json")
    assert np.array_equal(p2, pos) and np.array_equal(n2, nrm) and np.array_equal(a2, alb) and e2 == eye
    _same_frames(ctx, back, (p2, n2, a2, e2))
    ctx.close()
    back.close()


def test_grid_dump_sections_cpu(cpu_lib, tmp_path):
    """VOXELS alone: voxelized, not injected (build_mips is refused until a light comes);
    LEVEL0 alone: traceable at once, the voxel state untouched; PYRAMID needs LEVEL0; a
    section whose state is missing is refused at save."""
    from vct import VctError, dump, scenes
    ctx = _grid(cpu_lib)
    dump.save_grid(ctx, tmp_path / "v", level0=False)
    dump.save_grid(ctx, tmp_path / "l", voxels=False)
    with pytest.raises(VctError, match="PYRAMID needs"):
        dump.save_grid(ctx, tmp_path / "p", voxels=False, level0=False, pyramid=True)
    fresh = _ctx(cpu_lib, 16)
    with pytest.raises(VctError, match="ESTATE"):
        dump.save_grid(fresh, tmp_path / "x")
    v = dump.load_grid(tmp_path / "v", lib=cpu_lib)
    with pytest.raises(VctError, match="ESTATE"):
        v.build_mips()
    v.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    v.build_mips()
    _same_grids(ctx, v)
    lv = dump.load_grid(tmp_path / "l", lib=cpu_lib)
    _same_frames(ctx, lv, _gbuf(16))
    with pytest.raises(VctError, match="ESTATE"):
        lv.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)   # no voxels in that dump
    for x in (ctx, fresh, v, lv):
        x.close()


def test_grid_dump_damage_refused(cpu_lib, tmp_path):
    from vct import Context, dump
    ctx = _grid(cpu_lib)
    dump.save_grid(ctx, tmp_path / "g", pyramid=True)
    raw = bytearray((tmp_path / "g.bin").read_bytes())
    raw[100] ^= 1
    (tmp_path / "g.bin").write_bytes(bytes(raw))
    with pytest.raises(ValueError, match="sha256"):
        dump.load_grid(tmp_path / "g", lib=cpu_lib)
    (tmp_path / "g.bin").write_bytes(bytes(raw[:-4]))
    with pytest.raises(ValueError, match="length"):
        dump.load_grid(tmp_path / "g", lib=cpu_lib)
    with pytest.raises(ValueError, match="gbuffer"):
        dump.load_gbuffer(tmp_path / "g")
    hdr = (tmp_path / "g.json").read_text()
    (tmp_path / "bad.json").write_text(hdr.replace('"vct-dump/2"', '"vct-dump/9"'))
    with pytest.raises(ValueError, match="not a readable"):
        dump.load_grid(tmp_path / "bad", lib=cpu_lib)
    dump.save_grid(ctx, tmp_path / "h")
    other = Context(8, (0, 0, 0), 1.0, lib=cpu_lib)
    with pytest.raises(ValueError, match="context n=8"):
        dump.load_grid(tmp_path / "h", ctx=other)
    # same n and aniso, another placement: refused too, and the context is unchanged
    moved = Context(16, (0.5, 0, 0), ctx.extent, lib=cpu_lib)
    with pytest.raises(ValueError, match="aabb_min"):
        dump.load_grid(tmp_path / "h", ctx=moved)
    bigger = Context(16, ctx.aabb_min, ctx.extent * 2, lib=cpu_lib)
    with pytest.raises(ValueError, match="extent"):
        dump.load_grid(tmp_path / "h", ctx=bigger)
    iso = Context(16, ctx.aabb_min, ctx.extent, aniso=False, lib=cpu_lib)
    with pytest.raises(ValueError, match="aniso"):
        dump.load_grid(tmp_path / "h", ctx=iso)
    for x in (ctx, other, moved, bigger, iso):
        x.close()


def _failing_pyramid_dump(ctx, tmp_path):
    """A dump whose payload is intact (length and sha256 re-stamped) but whose last pyramid
    texel differs from the rebuilt one: refused only after the grid began to change."""
    import hashlib
    import json
    from vct import dump
    dump.save_grid(ctx, tmp_path / "f", pyramid=True)
    raw = bytearray((tmp_path / "f.bin").read_bytes())
    raw[-2] ^= 0x40                     # an exponent bit of the last float of the top level
    (tmp_path / "f.bin").write_bytes(bytes(raw))
    hdr = json.loads((tmp_path / "f.json").read_text())
    hdr["sha256"] = hashlib.sha256(bytes(raw)).hexdigest()
    (tmp_path / "f.json").write_text(json.dumps(hdr))
    return tmp_path / "f"


def _assert_load_fails_invalid(lib, tmp_path, n, name):
    """a load that fails after the header checks leaves no half-loaded grid:
    inject, mips and trace refuse the context (VCT_ESTATE) until a new voxelization."""
    from helpers import scene_arrays
    from vct import VctError, dump, scenes
    src = _grid(lib, n=n, name=name)
    bad = _failing_pyramid_dump(src, tmp_path)
    dst = _grid(lib, n=n, name=name, light=LIGHT2)
    with pytest.raises(ValueError, match="differ"):
        dump.load_grid(bad, ctx=dst)
    pos, nrm, alb, eye = _gbuf(n)
    with pytest.raises(VctError, match="ESTATE"):
        dst.trace(pos, nrm, alb, eye)
    with pytest.raises(VctError, match="ESTATE"):
        dst.build_mips()
    with pytest.raises(VctError, match="ESTATE"):
        dst.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    _, (v, i, m, k) = scene_arrays(name)     # a new voxelization makes it usable again
    dst.voxelize(v, i, m, k)
    dst.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    dst.build_mips()
    _same_frames(src, dst, _gbuf(n))
    src.close()
    dst.close()


def test_grid_dump_failed_load_invalidates_cpu(cpu_lib, tmp_path):
    _assert_load_fails_invalid(cpu_lib, tmp_path, 16, "cornell")


@pytest.mark.gpu
def test_grid_dump_failed_load_invalidates_gpu(gpu_ready, tmp_path):
    _assert_load_fails_invalid(None, tmp_path, 32, "cornell")


def test_sha256_matches_hashlib(cpu_lib, tmp_path):
    """The C SHA-256 of vct_dumpio.c (the header's payload hash) is hashlib's."""
    import hashlib
    import json
    from vct import dump
    ctx = _grid(cpu_lib, n=8)
    dump.save_grid(ctx, tmp_path / "g", pyramid=True)
    raw = (tmp_path / "g.bin").read_bytes()
    hdr = json.loads((tmp_path / "g.json").read_text())
    assert hdr["payload_bytes"] == len(raw) and hdr["sha256"] == hashlib.sha256(raw).hexdigest()
    assert hdr["format"] == "vct-dump/2" and hdr["sections"] == ["voxels", "level0", "pyramid"]
    ctx.close()


@pytest.mark.gpu
def test_grid_dump_relight_gpu(gpu_ready, tmp_path):
    """The relight case on the HIP library (64^3 atrium), composite included."""
    import torch

    def composite(b, c, gb):
        pos, nrm, alb, eye = gb
        h, w = pos.shape[:2]
        dev = torch.device("cuda")
        g = [torch.from_numpy(x).to(dev) for x in (pos, nrm, alb)]
        outs = []
        for ctx in (b, c):
            f = ctx.trace(pos, nrm, alb, eye)
            d, s = torch.from_numpy(f["diffuse"]).to(dev), torch.from_numpy(f["spec"]).to(dev)
            lin = torch.zeros((h, w, 4), device=dev)
            rgba = torch.zeros((h, w), dtype=torch.int32, device=dev)
            ctx.composite_device(*g, d, s, w, h, LIGHT2, out_linear4=lin, out_rgba8=rgba)
            torch.cuda.synchronize()
            outs.append((lin.cpu().numpy(), rgba.cpu().numpy()))
        assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    _relight_case(None, None, tmp_path, n=64, composite=composite)


@pytest.mark.gpu
def test_grid_dump_cross_backend(gpu_ready, cpu_lib, tmp_path):
    """One file format: a dump of the CPU backend relights on the HIP library and the
    other way round, to the same frames as a fresh context of the loading library."""
    for sub, (a, b) in {"c2g": (cpu_lib, None), "g2c": (None, cpu_lib)}.items():
        (tmp_path / sub).mkdir()
        _relight_case(a, b, tmp_path / sub, n=32)


@pytest.mark.gpu
def test_grid_dump_roundtrip_gpu(gpu_ready, tmp_path):
    """A grid dumped from the HIP library reloads to the same pyramid (verified against
    the dumped levels by vct_load_grid) and frame."""
    from vct import dump
    ctx = _grid(None, n=64, name="atrium")
    dump.save_grid(ctx, tmp_path / "g", pyramid=True)
    back = dump.load_grid(tmp_path / "g")
    _same_grids(ctx, back)
    _same_frames(ctx, back, _gbuf(ctx.n, 64, 48))
    ctx.close()
    back.close()
