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
    """Per-rank K4 driver: trace own tiles, all-gather, un-permute (torch + RCCL)."""

    def __init__(self, ctx, torch, dist, w: int, h: int, rank: int, world: int, device):
        self.ctx, self.torch, self.dist = ctx, torch, dist
        self.w, self.h, self.rank, self.world = w, h, rank, world
        self.max_tiles = tiles_for_rank(w, h, 0, world)
        npx = self.max_tiles * TILE * TILE
        f32 = torch.float32
        self.diff_c = torch.zeros((npx, 4), dtype=f32, device=device)
        self.spec_c = torch.zeros((npx, 4), dtype=f32, device=device)
        if world > 1:
            self.diff_g = torch.empty((world * npx, 4), dtype=f32, device=device)
            self.spec_g = torch.empty((world * npx, 4), dtype=f32, device=device)
        self.diff = torch.empty((h, w, 4), dtype=f32, device=device)
        self.spec = torch.empty((h, w, 4), dtype=f32, device=device)

    def trace_local(self, gb, eye, cone_steps=None, texel_fetches=None, steps_px=None, variant=0):
        pos, nrm, alb = gb
        self.ctx.trace_device(pos, nrm, alb, self.w, self.h, eye, self.diff_c, self.spec_c,
                              steps_px=steps_px, cone_steps=cone_steps, texel_fetches=texel_fetches,
                              tile_rank=self.rank, tile_world=self.world, tile_compact=True, variant=variant)

    def gather(self):
        if self.world > 1:
            if self.dist.get_backend() == "nccl":          # RCCL over xGMI
                self.dist.all_gather_into_tensor(self.diff_g, self.diff_c)
                self.dist.all_gather_into_tensor(self.spec_g, self.spec_c)
            else:                                          # gloo (CPU-side rehearsal of the same path)
                self.dist.all_gather(list(self.diff_g.chunk(self.world)), self.diff_c)
                self.dist.all_gather(list(self.spec_g.chunk(self.world)), self.spec_c)
            src_d, src_s = self.diff_g, self.spec_g
        else:
            src_d, src_s = self.diff_c, self.spec_c
        self.ctx.untile_device(src_d, self.w, self.h, self.world, self.diff)
        self.ctx.untile_device(src_s, self.w, self.h, self.world, self.spec)

    def frame(self, gb, eye, variant=0):
        self.trace_local(gb, eye, variant=variant)
        self.gather()
        return self.diff, self.spec
