"""Screen-tile partition of the cone-trace pass across ranks.

The framebuffer is cut into 64x64 tiles; tile t belongs to rank t % world
(interleaved, so background and early-out variance spread evenly).  Each rank
writes its tiles to a rank-compact buffer [max_tiles][64*64][4] (max_tiles =
tiles of rank 0, the largest share, so every rank's buffer has the same size
for all_gather); the all-gathered [world][max_tiles][64*64][4] buffer is
scattered back into the frame (vct_untile_device on the GPU, :func:`untile`
here on the host).

:class:`FrameTracer` is the per-rank driver bench.py uses: one process per GPU,
torch.distributed over RCCL ("nccl") for the level-0 grid broadcast and the
framebuffer all-gather.
"""
from __future__ import annotations

import numpy as np

TILE = 64


def num_tiles(w: int, h: int):
    tx, ty = (w + TILE - 1) // TILE, (h + TILE - 1) // TILE
    return tx, ty, tx * ty


def tiles_for_rank(w: int, h: int, rank: int, world: int) -> int:
    world = max(world, 1)
    _, _, total = num_tiles(w, h)
    if rank >= world or total <= rank:
        return 0
    return (total - rank + world - 1) // world


def compact_index(w: int, h: int, rank: int, world: int):
    """-> (frame_flat_idx, compact_flat_idx) of every in-frame pixel the rank owns."""
    tx, _, _ = num_tiles(w, h)
    nlt = tiles_for_rank(w, h, rank, world)
    lt = np.arange(nlt)
    t = lt * world + rank
    ox, oy = (t % tx) * TILE, (t // tx) * TILE
    py, px = np.meshgrid(np.arange(TILE), np.arange(TILE), indexing="ij")
    X = ox[:, None, None] + px[None]
    Y = oy[:, None, None] + py[None]
    cidx = (lt[:, None, None] * TILE * TILE + py[None] * TILE + px[None])
    m = (X < w) & (Y < h)
    return (Y * w + X)[m], cidx[m]


def pack(frame: np.ndarray, rank: int, world: int) -> np.ndarray:
    """[h][w][C] frame -> rank-compact [max_tiles*64*64][C] buffer (zeros off-frame)."""
    h, w = frame.shape[:2]
    maxt = tiles_for_rank(w, h, 0, world)
    out = np.zeros((maxt * TILE * TILE,) + frame.shape[2:], frame.dtype)
    fi, ci = compact_index(w, h, rank, world)
    out[ci] = frame.reshape((h * w,) + frame.shape[2:])[fi]
    return out


def untile(gathered: np.ndarray, w: int, h: int, world: int) -> np.ndarray:
    """[world][max_tiles*64*64][C] -> [h][w][C] (host mirror of vct_untile_device)."""
    C = gathered.shape[2:]
    out = np.zeros((h * w,) + C, gathered.dtype)
    for r in range(world):
        fi, ci = compact_index(w, h, r, world)
        out[fi] = gathered[r][ci]
    return out.reshape((h, w) + C)


class FrameTracer:
    """Per-rank K4 driver: trace own tiles, all-gather, un-permute (torch + RCCL).

    Each rank traces its tiles into one rank-compact buffer holding the diffuse
    and the specular plane side by side ([2][max_tiles*64*64][4]), so ONE
    all-gather moves both; one vct_untile_planes_device launch scatters them.
    With one rank there is nothing to exchange: the trace writes the frame.

    :meth:`frame` is one synchronous frame.  :meth:`step` / :meth:`drain` run
    frames as a pipeline (RCCL only): the all-gather of frame f runs on the
    process group's stream while frame f+1 is traced, and frame f is
    un-permuted after that trace was queued.  Two buffer sets alternate; the
    stream order (trace f+1, wait gather f, untile f, trace f+2, ...) keeps a
    buffer from being overwritten before its gather and untile have read it.
    """

    def __init__(self, ctx, torch, dist, w: int, h: int, rank: int, world: int, device):
        self.ctx, self.torch, self.dist = ctx, torch, dist
        self.w, self.h, self.rank, self.world = w, h, rank, world
        self.max_tiles = tiles_for_rank(w, h, 0, world)
        self.npx = self.max_tiles * TILE * TILE
        f32 = torch.float32
        nsets = 2 if world > 1 else 1
        self.comp = [torch.zeros((2, self.npx, 4), dtype=f32, device=device) for _ in range(nsets)]
        self.gath = [torch.empty((world, 2, self.npx, 4), dtype=f32, device=device) for _ in range(nsets)] \
            if world > 1 else []
        self.diff = torch.zeros((h, w, 4), dtype=f32, device=device)
        self.spec = torch.zeros((h, w, 4), dtype=f32, device=device)
        self.cur = 0
        self.pending = None

    def trace_local(self, gb, eye, cone_steps=None, texel_fetches=None, steps_px=None, variant=0, buf=0):
        pos, nrm, alb = gb
        if self.world == 1:      # the whole frame: straight into the outputs
            self.ctx.trace_device(pos, nrm, alb, self.w, self.h, eye, self.diff, self.spec,
                                  steps_px=steps_px, cone_steps=cone_steps, texel_fetches=texel_fetches,
                                  variant=variant)
            return
        c = self.comp[buf]
        self.ctx.trace_device(pos, nrm, alb, self.w, self.h, eye, c[0], c[1],
                              steps_px=steps_px, cone_steps=cone_steps, texel_fetches=texel_fetches,
                              tile_rank=self.rank, tile_world=self.world, tile_compact=True, variant=variant)

    def _pipelined(self):
        return self.world > 1 and self.dist.get_backend() == "nccl"

    def _gather(self, buf, async_op):
        if self.dist.get_backend() == "nccl":            # RCCL over xGMI
            return self.dist.all_gather_into_tensor(self.gath[buf], self.comp[buf], async_op=async_op)
        # gloo (CPU-side rehearsal of the same path)
        self.dist.all_gather(list(self.gath[buf].unbind(0)), self.comp[buf])
        return None

    def _untile(self, buf):
        self.ctx.untile_planes_device(self.gath[buf], self.w, self.h, self.world, (self.diff, self.spec))

    def gather(self, buf=0):
        if self.world > 1:
            self._gather(buf, False)
            self._untile(buf)

    def frame(self, gb, eye, variant=0):
        self.drain()
        self.trace_local(gb, eye, variant=variant)
        self.gather()
        return self.diff, self.spec

    def step(self, gb, eye, variant=0, on_traced=None):
        """One frame of the pipeline; the frame's outputs are complete after the next step() or drain()."""
        if not self._pipelined():
            self.trace_local(gb, eye, variant=variant)
            if on_traced:
                on_traced()
            self.gather()
            return
        b = self.cur
        self.cur ^= 1
        self.trace_local(gb, eye, variant=variant, buf=b)
        if on_traced:
            on_traced()
        work = self._gather(b, True)
        self.drain()
        self.pending = (work, b)

    def drain(self):
        if self.pending is not None:
            work, b = self.pending
            self.pending = None
            work.wait()                                     # current stream waits for the gather
            self._untile(b)
