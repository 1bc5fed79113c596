"""Grid / G-buffer dump and load (vct.dump, SURVEY.md §5 checkpoint / resume), on the CPU
backend of include/vct.h (oracle/_build/libvct_cpu.so; test infrastructure) and, marked
gpu, on the HIP library: a dumped grid reloads to the same pyramid and the same frame,
and a damaged dump is refused before anything is uploaded."""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def cpu_lib(oracle_mod):
    from vct import _lib
    return _lib.bind(C.CDLL(oracle_mod.CPU_BACKEND))


def _grid(lib, n=16, name="cornell"):
    from helpers import scene_arrays
    from vct import Context, scenes
    _, (v, i, m, k) = scene_arrays(name)
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E, lib=lib)
    ctx.voxelize(v, i, m, k)
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
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


@pytest.mark.parametrize("pyramid", [False, True])
def test_grid_dump_roundtrip_cpu(cpu_lib, tmp_path, pyramid):
    from vct import dump
    ctx = _grid(cpu_lib)
    dump.save_grid(ctx, tmp_path / "g", pyramid=pyramid)
    back = dump.load_grid(tmp_path / "g", lib=cpu_lib)
    assert (back.n, back.aniso, back.extent) == (ctx.n, ctx.aniso, ctx.extent)
    for a, b in zip(ctx.download_pyramid(), back.download_pyramid()):
        for fa, fb in zip(a, b):
            assert np.array_equal(fa, fb)
    pos, nrm, alb, eye = _gbuf(ctx.n)
    dump.save_gbuffer(tmp_path / "gb", pos, nrm, alb, eye)
    p2, n2, a2, e2 = dump.load_gbuffer(tmp_path / "gb.json")
    assert np.array_equal(p2, pos) and np.array_equal(n2, nrm) and np.array_equal(a2, alb) and e2 == eye
    f1, f2 = ctx.trace(pos, nrm, alb, eye), back.trace(p2, n2, a2, e2)
    for key in ("diffuse", "spec", "steps_px"):
        assert np.array_equal(f1[key], f2[key]), key
    ctx.close()
    back.close()


def test_grid_dump_damage_refused(cpu_lib, tmp_path):
    from vct import dump
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
    other = __import__("vct").Context(8, (0, 0, 0), 1.0, lib=cpu_lib)
    dump.save_grid(ctx, tmp_path / "h")
    with pytest.raises(ValueError, match="context n=8"):
        dump.load_grid(tmp_path / "h", ctx=other)
    ctx.close()
    other.close()


@pytest.mark.gpu
def test_grid_dump_roundtrip_gpu(gpu_ready, tmp_path):
    """A grid dumped from the HIP library reloads (upload + the deterministic K3) to the
    same pyramid (checked by load_grid's verify against the dumped levels) and frame."""
    from vct import dump
    ctx = _grid(None, n=64, name="atrium")
    dump.save_grid(ctx, tmp_path / "g", pyramid=True)
    back = dump.load_grid(tmp_path / "g", verify=True)
    pos, nrm, alb, eye = _gbuf(ctx.n, 64, 48)
    f1, f2 = ctx.trace(pos, nrm, alb, eye), back.trace(pos, nrm, alb, eye)
    for key in ("diffuse", "spec", "steps_px"):
        assert np.array_equal(f1[key], f2[key]), key
    ctx.close()
    back.close()
