"""The multi-rank arithmetic of the C-ABI RCCL path (include/vct.h vct_comm_*), on the CPU.

vct_comm_trace_frame places every rank's tiles in an exchange buffer laid out by
vct_comm_frame_layout (packed toward a presenting root, padded for VCT_ALL_RANKS);
the root un-permutes it.  With one GPU per test box no multi-rank RCCL run is
possible here, so this checks the same arithmetic without a collective: for 2, 3
and 8 ranks, every rank's compact tiles are placed where the layout says (as the
send/recv or all-gather would deliver them), and the frame is un-permuted by the C
library (the CPU backend's vct_untile_planes_*) and by the host mirror vct.multi.
Both libraries' layouts must agree with vct.multi's tile_offset / tiles_for_rank.
Also: the communicator-id exchange over a gloo group and the error codes.
"""
import ctypes as C
import os

import numpy as np
import pytest

from vct import VCT_ALL_RANKS, VctError, comm_frame_layout
from vct import multi as M

SIZES = [(1920, 1080), (200, 130), (64, 64), (65, 1)]


@pytest.fixture(scope="module")
def libs(oracle_mod):
    from vct import _lib
    return {"hip": _lib.load(), "cpu": _lib.bind(C.CDLL(oracle_mod.CPU_BACKEND))}


def _expected(w, h, R, r, root):
    maxt = M.tiles_for_rank(w, h, 0, R)
    mine = M.tiles_for_rank(w, h, r, R)
    _, _, T = M.num_tiles(w, h)
    if root == VCT_ALL_RANKS:
        return dict(buffer_tiles=R * 2 * maxt, diffuse_tile=r * 2 * maxt, spec_tile=r * 2 * maxt + maxt, tiles=mine,
                    exchange_tiles=2 * maxt)
    off = 2 * M.tile_offset(w, h, r, R)
    return dict(buffer_tiles=2 * T, diffuse_tile=off, spec_tile=off + mine, tiles=mine, exchange_tiles=2 * mine)


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("R", [1, 2, 3, 8])
def test_layout_matches_host_mirror(libs, w, h, R):
    for root in sorted({0, R - 1, VCT_ALL_RANKS}):
        for r in range(R):
            exp = _expected(w, h, R, r, root)
            for name, lib in libs.items():
                assert comm_frame_layout(w, h, R, r, root, lib) == exp, (name, root, r)


@pytest.mark.parametrize("w,h", SIZES[:3])
@pytest.mark.parametrize("R", [2, 3, 8])
def test_exchange_assembles_frame(libs, w, h, R):
    """Place each rank's compact tiles as the layout says, un-permute: the frame comes back."""
    rng = np.random.default_rng(R * 1000 + w)
    fd = rng.standard_normal((h, w, 4)).astype(np.float32)
    fs = rng.standard_normal((h, w, 4)).astype(np.float32)
    tpx = M.TILE * M.TILE
    cpu = libs["cpu"]
    for root in (0, R - 1, VCT_ALL_RANKS):
        L0 = comm_frame_layout(w, h, R, 0, root, cpu)
        buf = np.full((L0["buffer_tiles"] * tpx, 4), np.nan, np.float32)
        for r in range(R):
            L = comm_frame_layout(w, h, R, r, root, cpu)
            if L["tiles"] == 0:
                continue
            fi, ci = M.compact_index(w, h, r, R)
            plane = L["exchange_tiles"] // 2
            for frame, first in ((fd, L["diffuse_tile"]), (fs, L["spec_tile"])):
                blk = np.zeros((plane * tpx, 4), np.float32)
                blk[ci] = frame.reshape(-1, 4)[fi]
                buf[first * tpx:(first + plane) * tpx] = blk
        packed = root != VCT_ALL_RANKS
        # host mirror
        if packed:
            got = M.untile_packed(buf, w, h, R, 2)
        else:
            gg = buf.reshape(R, 2, -1, 4)
            got = [M.untile(gg[:, p], w, h, R) for p in range(2)]
        assert np.array_equal(got[0], fd) and np.array_equal(got[1], fs), (root, "mirror")
        # the C untile of the CPU backend (same entry points as the HIP library's)
        outs = [np.zeros((h, w, 4), np.float32) for _ in range(2)]
        arr = (C.c_void_p * 2)(*[o.ctypes.data for o in outs])
        fn = cpu.vct_untile_planes_packed_device if packed else cpu.vct_untile_planes_device
        from vct import Context
        ctx = Context(16, (0, 0, 0), 1.0, lib=cpu)
        assert fn(ctx.h, buf.ctypes.data, 2, w, h, R, C.cast(arr, C.c_void_p)) == 0
        ctx.close()
        assert np.array_equal(outs[0], fd) and np.array_equal(outs[1], fs), (root, "C untile")


def test_layout_errors(libs):
    for lib in libs.values():
        for args in ((0, 10, 2, 0, 0), (10, 10, 0, 0, 0), (10, 10, 2, 2, 0), (10, 10, 2, 0, 2), (10, 10, 2, 0, -5)):
            with pytest.raises(VctError, match="EINVAL"):
                comm_frame_layout(*args, lib=lib)


def test_cpu_backend_comm_errors(libs):
    from vct import Context
    cpu = libs["cpu"]
    ctx = Context(16, (0, 0, 0), 1.0, lib=cpu)
    with pytest.raises(VctError, match="ESTATE"):
        ctx.comm_synchronize()
    with pytest.raises(VctError, match="EINVAL"):
        ctx.comm_set_timeout(0)
    cid = Context.comm_get_id(cpu)
    with pytest.raises(VctError, match="ECOMM"):       # the CPU backend has no RCCL: one rank only
        ctx.comm_init(cid, 2, 0)
    ctx.comm_init(cid, 1, 0)
    ctx.comm_set_timeout(5000)
    ctx.comm_synchronize()
    ctx.comm_destroy()
    ctx.close()


def _id_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    made = bytes(range(128)) if rank == 0 else None
    got = M.share_comm_id(dist, rank, get_id=(lambda: made) if rank == 0 else None)
    q.put((rank, got))
    dist.destroy_process_group()


def test_comm_id_shared_over_gloo():
    """vct.multi.share_comm_id: rank 0's 128-byte ncclUniqueId reaches every rank."""
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_id_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert all(res[r] == bytes(range(128)) for r in range(3))
