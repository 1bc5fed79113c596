"""The boundary on the CPU: include/vct.h implemented by the oracle
(oracle/_build/libvct_cpu.so, SURVEY.md 8b "one .so per backend"; test
infrastructure, never loaded by the product).

The same vct.Context binding drives it, so these tests check, without a GPU,
that the ABI's call sequence, state machine and error codes behave as the HIP
library's (tests/test_parity_gpu.py::test_backends_agree compares the two
libraries call for call on the GPU box), and that the host-side pieces around
the kernels (tile partition, compact layout, un-permute) compose to the
single-rank frame.
"""
import ctypes as C

import numpy as np
import pytest

from test_abi import declared_functions


@pytest.fixture(scope="module")
def cpu_lib(oracle_mod):
    from vct import _lib
    return _lib.bind(C.CDLL(oracle_mod.CPU_BACKEND))


def _ptr(a):
    return a.ctypes.data


def _ctx(cpu_lib, n=32, name="atrium", **kw):
    from helpers import scene_arrays
    from vct import Context, scenes
    s, (v, i, m, k) = scene_arrays(name)
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E, lib=cpu_lib, **kw)
    ctx.voxelize(v, i, m, k)
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ctx.build_mips()
    return ctx, s, (v, i, m, k), (g0, E)


def test_cpu_backend_exports_the_header(oracle_mod):
    import re
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", oracle_mod.CPU_BACKEND], capture_output=True,
                         text=True).stdout
    exported = set(re.findall(r"\bT (vct_[a-z0-9_]+)", out))
    assert set(declared_functions()) <= exported


def test_pipeline_equals_oracle(cpu_lib, oracle_mod):
    from vct import scenes
    from vct.camera import Camera
    ctx, s, (v, i, m, k), (g0, E) = _ctx(cpu_lib)
    ref = oracle_mod.pipeline(32, g0, E, v, i, m, k, scenes.LIGHT_DIR)
    sums, counts = ctx.download_accum()
    assert np.array_equal(sums, ref["sums"]) and np.array_equal(counts, ref["counts"])
    assert np.array_equal(ctx.download_level(0), ref["r0"])
    cam = Camera()
    pos, nrm, alb = scenes.raycast_numpy(s, cam, 48, 32)
    out = ctx.trace(pos, nrm, alb, cam.position)
    tr = oracle_mod.trace(32, g0, E, ref["r0"], ref["pyr"], pos, nrm, alb, cam.position)
    assert np.array_equal(out["diffuse"], tr["diffuse"]) and np.array_equal(out["spec"], tr["spec"])
    assert out["cone_steps"] == tr["cone_steps"] and np.array_equal(out["steps_px"], tr["steps_px"])
    ctx.close()


def test_gbuffer_caster_close_to_numpy(cpu_lib):
    """The float32 caster (the HIP caster's restatement) against the float64 numpy cast."""
    from vct import scenes
    from vct.camera import Camera
    ctx, s, _, _ = _ctx(cpu_lib, 16)
    cam = Camera()
    w, h = 64, 40
    bufs = [np.zeros((h, w, 4), np.float32) for _ in range(3)]
    ctx.gbuffer_raycast_device(cam, w, h, 0.1, *[_ptr(b) for b in bufs])
    rp, rn, ra = scenes.raycast_numpy(s, cam, w, h, 0.1)
    assert (bufs[0][..., 3] == rp[..., 3]).mean() > 0.995
    both = (bufs[0][..., 3] > 0) & (rp[..., 3] > 0)
    assert np.abs(bufs[0][both][:, :3] - rp[both][:, :3]).max() < 1e-3
    raster = [np.zeros_like(b) for b in bufs]
    ctx.gbuffer_raster_device(cam, w, h, 0.1, *[_ptr(b) for b in raster])
    assert all(np.array_equal(a, b) for a, b in zip(bufs, raster))
    ctx.close()


@pytest.mark.parametrize("world", [2, 3])
def test_tiles_compact_untile_equal_full_frame(cpu_lib, world):
    from vct import scenes
    from vct.camera import Camera
    from vct.multi import tiles_for_rank
    ctx, s, _, _ = _ctx(cpu_lib, 16)
    cam = Camera()
    w, h = 130, 70
    gb = [np.zeros((h, w, 4), np.float32) for _ in range(3)]
    ctx.gbuffer_raycast_device(cam, w, h, scenes.ROUGHNESS, *[_ptr(b) for b in gb])
    d, sp = np.zeros((h, w, 4), np.float32), np.zeros((h, w, 4), np.float32)
    cnt = np.zeros(1, np.int64)
    ctx.trace_device(*[_ptr(b) for b in gb], w, h, cam.position, _ptr(d), _ptr(sp), cone_steps=_ptr(cnt))
    maxt = tiles_for_rank(w, h, 0, world)
    assert ctx.lib.vct_tiles_for_rank(w, h, 0, world) == maxt
    g = np.zeros((world, 2, maxt * 4096, 4), np.float32)
    tot = np.zeros(1, np.int64)
    for r in range(world):
        ctx.trace_device(*[_ptr(b) for b in gb], w, h, cam.position, _ptr(g[r, 0]), _ptr(g[r, 1]),
                         cone_steps=_ptr(tot), tile_rank=r, tile_world=world, tile_compact=True)
    assert tot[0] == cnt[0] > 0
    fd, fs = np.zeros_like(d), np.zeros_like(sp)
    ctx.untile_planes_device(_ptr(g), w, h, world, (_ptr(fd), _ptr(fs)))
    assert np.array_equal(fd, d) and np.array_equal(fs, sp)
    ctx.close()


def test_state_machine_and_errors(cpu_lib):
    """The same status codes as the HIP library's test_abi_errors."""
    from vct import Context, VctError, scenes
    from vct._lib import VctConfig, VctTraceArgs
    cfg = VctConfig()
    cfg.n, cfg.extent, cfg.n_diffuse = 24, 1.0, 9
    h = C.c_void_p()
    assert cpu_lib.vct_create(C.byref(cfg), C.byref(h)) == 1                 # EINVAL: n not 2^k
    cfg.n, cfg.n_diffuse = 16, 7
    assert cpu_lib.vct_create(C.byref(cfg), C.byref(h)) == 1                 # EINVAL: cone count
    g0, E = scenes.grid_for_unit_box(16)
    ctx = Context(16, g0, E, lib=cpu_lib)
    with pytest.raises(VctError, match="ESTATE"):
        ctx.inject_directional((0, 1, 0))                                    # before voxelize
    with pytest.raises(VctError, match="ESTATE"):
        ctx.build_mips()                                                     # before inject
    pos = np.zeros((4, 4, 4), np.float32)
    with pytest.raises(VctError, match="ESTATE"):
        ctx.trace(pos, pos, pos, (0, 0, 3))                                  # before mips
    with pytest.raises(VctError, match="EINVAL"):
        ctx.voxelize(np.zeros((3, 14), np.float32), np.array([0, 1, 5], np.uint32))   # index out of range
    ctx.voxelize(np.zeros((3, 14), np.float32), np.array([0, 1, 2], np.uint32))
    with pytest.raises(VctError, match="EINVAL"):
        ctx.inject_directional((0, 0, 0))                                    # zero light direction
    ctx.inject_directional((0, 1, 0))
    ctx.build_mips()
    a = VctTraceArgs()
    buf = np.zeros(64 * 4 + 8, np.float32)
    base = _ptr(buf) + (16 - _ptr(buf) % 16) % 16
    a.pos4 = a.nrm4 = a.alb4 = a.diffuse4 = a.spec4 = base
    a.width = a.height = 2
    a.tile_world, a.tile_rank = 2, 2
    assert cpu_lib.vct_trace_device(ctx.h, C.byref(a)) == 1                  # tile_rank >= tile_world
    a.tile_world = a.tile_rank = 0
    a.cone_steps = base + 4
    assert cpu_lib.vct_trace_device(ctx.h, C.byref(a)) == 1                  # misaligned counter
    a.cone_steps = None
    a.pos4 = base + 4
    assert cpu_lib.vct_trace_device(ctx.h, C.byref(a)) == 1                  # misaligned G-buffer
    with pytest.raises(VctError, match="EINVAL"):
        ctx.download_level(1, 6)                                             # face out of range
    ctx.close()


def test_multi_device_context_cpu(cpu_lib, oracle_mod):
    """vct_create_multi on the CPU backend: the same call sequence and status codes as
    the HIP library (test_parity_gpu.py::test_multi_device_context); the CPU traces
    every rank's tiles itself, so the frame equals the single-device one."""
    from vct._lib import VctConfig, VctTraceArgs
    cfg = VctConfig()
    cfg.n, cfg.extent, cfg.n_diffuse = 16, 1.0, 9
    h = C.c_void_p()
    assert cpu_lib.vct_create_multi(C.byref(cfg), 0, C.byref(h)) == 1       # EINVAL: no device
    assert cpu_lib.vct_create_multi(C.byref(cfg), 65, C.byref(h)) == 1      # EINVAL: too many
    one, s, _, (g0, E) = _ctx(cpu_lib, 16)
    multi, _, _, _ = _ctx(cpu_lib, 16, devices=3)
    assert (one.num_devices, multi.num_devices) == (1, 3)
    from vct.camera import Camera
    from vct import scenes
    cam = Camera()
    pos, nrm, alb = scenes.raycast_numpy(s, cam, 40, 24)
    a, b = one.trace(pos, nrm, alb, cam.position), multi.trace(pos, nrm, alb, cam.position)
    for key in ("diffuse", "spec", "steps_px"):
        assert np.array_equal(a[key], b[key]), key
    args = VctTraceArgs()
    buf = np.zeros(64 * 4 + 8, np.float32)
    base = _ptr(buf) + (16 - _ptr(buf) % 16) % 16
    args.pos4 = args.nrm4 = args.alb4 = args.diffuse4 = args.spec4 = base
    args.width = args.height = 2
    args.tile_world, args.tile_rank = 2, 0
    assert cpu_lib.vct_trace_device(multi.h, C.byref(args)) == 1            # the context splits itself
    assert cpu_lib.vct_trace_device(one.h, C.byref(args)) == 0
    multi.close()
    one.close()


def test_partial_grid_after_bad_indices_is_refused(cpu_lib):
    """A voxelization that fails on out-of-range indices leaves no usable grid:
    inject after it is VCT_ESTATE (the HIP library's rule too, test_parity_gpu)."""
    from vct import Context, VctError, scenes
    g0, E = scenes.grid_for_unit_box(16)
    ctx = Context(16, g0, E, lib=cpu_lib)
    v = np.zeros((3, 14), np.float32)
    ctx.voxelize(v, np.array([0, 1, 2], np.uint32))
    with pytest.raises(VctError, match="EINVAL"):
        ctx.voxelize(v, np.array([0, 1, 5], np.uint32))
    with pytest.raises(VctError, match="ESTATE"):
        ctx.inject_directional((0, 1, 0))
    ctx.voxelize(v, np.array([0, 1, 2], np.uint32))      # a good call restores the state
    ctx.inject_directional((0, 1, 0))


def test_host_argument_checks(cpu_lib):
    """Python-side length / shape contracts of vct_voxelize (tri_material has n_idx / 3
    entries, kd4 is [materials, 4]) are enforced before the C call."""
    from vct import Context, VctError, scenes
    g0, E = scenes.grid_for_unit_box(16)
    ctx = Context(16, g0, E, lib=cpu_lib)
    v = np.zeros((6, 14), np.float32)
    idx = np.arange(6, dtype=np.uint32)
    with pytest.raises(VctError, match="EINVAL.*tri_material"):
        ctx.voxelize(v, idx, np.zeros(1, np.uint32), np.ones((1, 4), np.float32))
    with pytest.raises(VctError, match="EINVAL.*kd4"):
        ctx.voxelize(v, idx, np.zeros(2, np.uint32), np.ones(4, np.float32))
    with pytest.raises(VctError, match="EINVAL.*multiple of 3"):
        ctx.voxelize(v, idx[:4])
    ctx.voxelize(v, idx, np.zeros(2, np.uint32), np.ones((1, 4), np.float32))


class _FakeDeviceTensor:
    """Just enough of a torch CUDA tensor for Context._dev's checks."""

    def __init__(self, numel, dtype="torch.float32", index=0, contiguous=True, cuda=True, shape=None):
        self.is_cuda = cuda
        self.shape = shape or (numel,)
        self.dtype = dtype
        self._n, self._c = numel, contiguous
        self.device = type("D", (), {"index": index, "__str__": lambda s: f"cuda:{index}"})()

    def is_contiguous(self):
        return self._c

    def dim(self):
        return len(self.shape)

    def numel(self):
        return self._n

    def data_ptr(self):
        return 0x1000


def test_device_pointer_checks(cpu_lib):
    """Context._dev refuses host tensors, the wrong device / dtype, non-contiguous and
    undersized buffers before a pointer reaches the C-ABI (a host pointer or a short
    output would fault or overrun the GPU); 64-bit indices are refused for K1."""
    import torch
    from vct import Context, VctError, scenes
    g0, E = scenes.grid_for_unit_box(16)
    ctx = Context(16, g0, E, lib=cpu_lib, device=0)
    F = _FakeDeviceTensor
    assert ctx._dev(F(64), "x", min_numel=64) == 0x1000
    assert ctx._dev(None, "x") is None and ctx._dev(1234, "x") == 1234
    with pytest.raises(VctError, match="EINVAL.*device .cuda. tensor"):
        ctx._dev(torch.zeros(64), "x")
    with pytest.raises(VctError, match="EINVAL.*context on device 0"):
        ctx._dev(F(64, index=1), "x")
    with pytest.raises(VctError, match="EINVAL.*dtype"):
        ctx._dev(F(64, dtype="torch.float64"), "x")
    with pytest.raises(VctError, match="EINVAL.*contiguous"):
        ctx._dev(F(64, contiguous=False), "x")
    with pytest.raises(VctError, match="EINVAL.*at least 65"):
        ctx._dev(F(64), "x", min_numel=65)
    # trace_device sizes every buffer from the frame (compact: the rank's tiles)
    w, h = 100, 70
    gb = [F(4 * w * h) for _ in range(3)]
    with pytest.raises(VctError, match="EINVAL.*diffuse4"):
        ctx.trace_device(*gb, w, h, (0, 0, 3), F(4 * w * h - 1), F(4 * w * h))
    with pytest.raises(VctError, match="EINVAL.*steps_px.*dtype"):
        ctx.trace_device(*gb, w, h, (0, 0, 3), F(4 * w * h), F(4 * w * h), steps_px=F(w * h))
    with pytest.raises(VctError, match="EINVAL.*diffuse4"):
        ctx.trace_device(*gb, w, h, (0, 0, 3), F(4 * 4096 - 4), F(4 * 4096), tile_rank=1, tile_world=2,
                         tile_compact=True)
    with pytest.raises(VctError, match="EINVAL.*64-bit"):
        ctx.voxelize_device(F(14 * 3, shape=(3, 14)), F(3, dtype="torch.int64"))
    # the C-ABI bounds kd4 and the material map by one n_mat: a map longer than kd4 is
    # refused (K1 would read kd4 past its end on the device), as on the host path
    with pytest.raises(VctError, match="EINVAL.*material_map has 3 entries for 2 materials"):
        ctx.voxelize_device(F(14 * 3, shape=(3, 14)), F(3, dtype="torch.int32"), F(1, dtype="torch.int32"),
                            F(8, shape=(2, 4)), material_map=F(3, dtype="torch.int32"))


def test_comm_one_rank(cpu_lib):
    """vct_comm_* on the CPU backend: a one-rank group runs a host's call sequence
    unchanged (the HIP library runs the same sequence over RCCL on the GPU box)."""
    from vct import VCT_ALL_RANKS, Context, VctError, scenes
    from vct.camera import Camera
    ctx, s, _, (g0, E) = _ctx(cpu_lib, n=16)
    cid = Context.comm_get_id(cpu_lib)
    assert len(cid) == 128
    with pytest.raises(VctError, match="ECOMM"):
        ctx.comm_init(cid, 2, 0)
    ctx.comm_init(cid, 1, 0)
    ctx.comm_broadcast_level0(0)
    ctx.build_mips()
    cam = Camera()
    w, h = 48, 32
    gb = scenes.raycast_numpy(s, cam, w, h)
    d, sp = np.zeros((h, w, 4), np.float32), np.zeros((h, w, 4), np.float32)
    ctx.comm_trace_frame(*[_ptr(b) for b in gb], w, h, cam.position, _ptr(d), _ptr(sp), root=VCT_ALL_RANKS)
    ref = ctx.trace(*gb, cam.position)
    assert np.array_equal(d, ref["diffuse"]) and np.array_equal(sp, ref["spec"])
    ctx.comm_destroy()


def test_upload_level0_refuses_non_finite(cpu_lib):
    """K4 composites branch-free (a finished lane adds fmaf(+0, sample, c)), which needs
    finite radiance: vct_upload_level0 refuses Inf / NaN (both libraries check it on the
    host, before any device work)."""
    from vct import Context, VctError
    ctx = Context(8, (0, 0, 0), 1.0, lib=cpu_lib)
    r0 = np.zeros((8, 8, 8, 4), np.float32)
    ctx.upload_level0(r0)
    for bad in (np.inf, -np.inf, np.nan):
        r = r0.copy()
        r[3, 4, 5, 1] = bad
        with pytest.raises(VctError, match="EINVAL"):
            ctx.upload_level0(r)
    ctx.close()
