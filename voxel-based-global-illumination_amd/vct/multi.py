"""Screen-tile partition of the cone-trace pass across ranks.

The framebuffer is cut into 64x64 tiles; tile t belongs to rank t % world
(interleaved, so background and early-out variance spread evenly).  Each rank
writes its tiles to a rank-compact buffer, and the frame is assembled from the
ranks' buffers in one of two ways:

* ``present`` (default): every rank sends exactly its own tiles to the
  presenting rank (RCCL send / recv; each rank's bytes cross its own xGMI
  link once), which un-permutes the packed buffer (rank r's
  [planes][tiles(r)*64*64] block at tile offset planes * tile_offset(r)).
  Only the presenting rank holds the frame, as a renderer presents from one
  GPU.
* ``allgather`` (the north_star collective): rank buffers padded to rank 0's
  share ([max_tiles][64*64][4]) are all-gathered, and every rank un-permutes
  the whole [world][planes][max_tiles*64*64] buffer.

vct_untile_planes(_packed)_device does the un-permute on the GPU;
:func:`untile` / :func:`untile_packed` are the host mirrors.

:class:`FrameTracer` is the per-rank driver bench.py uses: one process per GPU,
torch.distributed over RCCL ("nccl") for the level-0 grid broadcast and the
frame exchange.
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


def tile_offset(w: int, h: int, rank: int, world: int) -> int:
    """Tiles of ranks 0..rank-1: rank * q + min(rank, T mod world) (vct_tile_offset)."""
    world = max(world, 1)
    _, _, total = num_tiles(w, h)
    q, rem = divmod(total, world)
    return 0 if rank >= world else rank * q + min(rank, rem)


def untile_packed(packed: np.ndarray, w: int, h: int, world: int, planes: int) -> list:
    """Packed [sum_r planes*tiles(r)*64*64][C] -> planes x [h][w][C] (host mirror of
    vct_untile_planes_packed_device)."""
    C = packed.shape[1:]
    outs = [np.zeros((h * w,) + C, packed.dtype) for _ in range(planes)]
    for r in range(world):
        fi, ci = compact_index(w, h, r, world)
        base, nt = planes * tile_offset(w, h, r, world), tiles_for_rank(w, h, r, world)
        for p in range(planes):
            outs[p][fi] = packed[(base + p * nt) * TILE * TILE + ci]
    return [o.reshape((h, w) + C) for o in outs]


def untile(gathered: np.ndarray, w: int, h: int, world: int) -> np.ndarray:
    """[world][max_tiles*64*64][C] -> [h][w][C] (host mirror of vct_untile_device)."""
    C = gathered.shape[2:]
    out = np.zeros((h * w,) + C, gathered.dtype)
    for r in range(world):
        fi, ci = compact_index(w, h, r, world)
        out[fi] = gathered[r][ci]
    return out.reshape((h, w) + C)


class FrameTracer:
    """Per-rank K4 driver: trace own tiles, exchange, un-permute (torch + RCCL).

    mode "present": rank r traces its tiles into [2][tiles(r)*64*64][4]
    (diffuse plane, then specular plane) and sends exactly that to the
    presenting rank `root`, which traces its own tiles straight into its slice
    of the packed receive buffer; one packed two-plane untile assembles the
    frame on `root` only.  mode "allgather": buffers padded to rank 0's share,
    ONE all-gather moves both planes to every rank, one two-plane untile each.
    With one rank there is nothing to exchange: the trace writes the frame.

    :meth:`frame` is one synchronous frame.  :meth:`step` / :meth:`drain` run
    frames as a pipeline; a step's outputs are complete (on the caller's
    current stream) after the next step() or drain().  Two buffer sets
    alternate.  With `overlap` frame f is traced on trace stream f % 2, so the
    trace of frame f+1 starts while the last waves of frame f drain (a K4 launch
    ends in a tail of few busy CUs) and, over RCCL, the exchange of frame f
    (issued on the trace stream, so it waits for that trace only) runs beside
    the trace of frame f+1.  Buffer set b is reused by frame f+2 only after the
    caller's stream has un-permuted frame f (the trace stream waits for the
    caller's stream first).  Without overlap the same order runs on one stream:
    trace f+1, wait exchange f, untile f, trace f+2, ...

    Whether overlap pays depends on the launch and on the hardware queues the
    two streams land on, so `overlap=None` (default, one rank or an RCCL group
    on a GPU) decides by timing: :meth:`tune` runs 16 pipelined frames on one
    stream and on two stream pairs (normal and high priority) and keeps the
    fastest overlap if it is 1.5 % faster; an untuned tracer tunes on its first
    step().  Measured on one MI355X: 1080p full frame 1.170 -> 1.127 ms, a
    rank's launch of an 8-rank split 0.243 -> 0.172 ms, 4K 4.97 -> 4.82 ms.
    """

    def __init__(self, ctx, torch, dist, w: int, h: int, rank: int, world: int, device, mode: str = "present",
                 root: int = 0, overlap=None):
        if mode not in ("present", "allgather"):
            raise ValueError(f"mode {mode!r}: 'present' or 'allgather'")
        self.ctx, self.torch, self.dist = ctx, torch, dist
        self.w, self.h, self.rank, self.world = w, h, rank, world
        self.mode, self.root = mode, root
        self.device = torch.device(device)
        self.max_tiles = tiles_for_rank(w, h, 0, world)
        self.my_tiles = tiles_for_rank(w, h, rank, world)
        _, _, self.total_tiles = num_tiles(w, h)
        gpu = self.device.type == "cuda"
        can = gpu and (world == 1 or self._nccl())
        if overlap and not can:
            raise ValueError("overlap: needs a GPU device and one rank or an RCCL group")
        self.auto = overlap is None and can          # decided by tune()
        self.tuned = None
        self.overlap = bool(overlap)
        two = can and overlap is not False
        self.streams = [torch.cuda.Stream(self.device) for _ in range(2)] if two else None
        f32 = torch.float32
        nsets = 2 if (world > 1 or two) else 1
        tpx = TILE * TILE
        self.comp, self.gath = [], []
        if world > 1 and mode == "allgather":
            self.npx = self.max_tiles * tpx
            self.comp = [torch.zeros((2, self.npx, 4), dtype=f32, device=device) for _ in range(nsets)]
            self.gath = [torch.empty((world, 2, self.npx, 4), dtype=f32, device=device) for _ in range(nsets)]
        elif world > 1:
            self.npx = self.my_tiles * tpx
            if rank == root:     # packed receive buffer; the root's own slice is its trace target
                self.gath = [torch.zeros((2 * self.total_tiles * tpx, 4), dtype=f32, device=device)
                             for _ in range(nsets)]
                off = 2 * tile_offset(w, h, rank, world) * tpx
                self.comp = [g[off:off + 2 * self.npx].view(2, self.npx, 4) for g in self.gath]
            else:
                self.comp = [torch.zeros((2, self.npx, 4), dtype=f32, device=device) for _ in range(nsets)]
        # one rank: the frames themselves alternate (the trace writes them)
        self.outs = [(torch.zeros((h, w, 4), dtype=f32, device=device),
                      torch.zeros((h, w, 4), dtype=f32, device=device)) for _ in range(nsets if world == 1 else 1)]
        self._set = 0            # the set holding the latest retired frame (one rank)
        self._ready = None       # its completion event, waited for when it is read (one rank, overlap)
        self.nsets = nsets
        self.cur = 0
        self.pending = None
        self._ops = {}           # "present" P2P descriptors per buffer set (_p2p_ops)

    def _order_reads(self):
        if self._ready is not None:
            self.torch.cuda.current_stream(self.device).wait_event(self._ready)
            self._ready = None

    @property
    def diff(self):
        """Diffuse + AO of the latest completed frame, ordered on the caller's current stream."""
        self._order_reads()
        return self.outs[self._set if self.world == 1 else 0][0]

    @property
    def spec(self):
        """Specular of the latest completed frame, ordered on the caller's current stream."""
        self._order_reads()
        return self.outs[self._set if self.world == 1 else 0][1]

    @property
    def holds_frame(self) -> bool:
        """True where the assembled frame lands (every rank for allgather)."""
        return self.world == 1 or self.mode == "allgather" or self.rank == self.root

    def trace_local(self, gb, eye, cone_steps=None, texel_fetches=None, steps_px=None, variant=0, buf=0):
        pos, nrm, alb = gb
        if self.world == 1:      # the whole frame: straight into the outputs of set `buf`
            d, s = self.outs[buf]
            self.ctx.trace_device(pos, nrm, alb, self.w, self.h, eye, d, s,
                                  steps_px=steps_px, cone_steps=cone_steps, texel_fetches=texel_fetches,
                                  variant=variant)
            return
        if self.my_tiles == 0:
            return
        c = self.comp[buf]
        self.ctx.trace_device(pos, nrm, alb, self.w, self.h, eye, c[0], c[1],
                              steps_px=steps_px, cone_steps=cone_steps, texel_fetches=texel_fetches,
                              tile_rank=self.rank, tile_world=self.world, tile_compact=True, variant=variant)

    def local_planes(self, buf=0):
        """(diffuse, spec) as trace_local(buf=buf) writes them: the frame (one rank) or this
        rank's compact tiles; None for a rank without tiles."""
        if self.world == 1:
            return self.outs[buf]
        if self.my_tiles == 0:
            return None
        return self.comp[buf][0], self.comp[buf][1]

    @property
    def last_buf(self):
        """The buffer set of the latest frame traced by step() / frame()."""
        return (self.cur - 1) % self.nsets if self._pipelined() else 0

    def _nccl(self):
        return self.world > 1 and self.dist.get_backend() == "nccl"

    def _pipelined(self):
        return self.overlap or self._nccl()

    def _exchange(self, buf, async_op):
        """Moves frame `buf`'s tiles; returns the outstanding works (async RCCL) or []."""
        d = self.dist
        if self.mode == "allgather":
            if self._nccl():                                 # RCCL over xGMI
                w = d.all_gather_into_tensor(self.gath[buf], self.comp[buf], async_op=async_op)
                return [w] if async_op else []
            d.all_gather(list(self.gath[buf].unbind(0)), self.comp[buf])   # gloo (CPU rehearsal)
            return []
        ops = self._p2p_ops(buf)
        if not ops:
            return []
        works = d.batch_isend_irecv(ops)
        if not async_op:
            for w in works:
                w.wait()
            return []
        return works

    def _p2p_ops(self, buf):
        """The "present" exchange of buffer set `buf` as P2P op descriptors, built once per
        set (the root's receive list is the per-frame host cost that grows with the ranks)."""
        if buf not in self._ops:
            d, tpx = self.dist, TILE * TILE
            ops = []
            if self.rank == self.root:
                for r in range(self.world):
                    nt = tiles_for_rank(self.w, self.h, r, self.world)
                    if r == self.root or nt == 0:
                        continue
                    off = 2 * tile_offset(self.w, self.h, r, self.world) * tpx
                    ops.append(d.P2POp(d.irecv, self.gath[buf][off:off + 2 * nt * tpx], r))
            elif self.my_tiles:
                ops.append(d.P2POp(d.isend, self.comp[buf].view(-1, 4), self.root))
            self._ops[buf] = ops
        return self._ops[buf]

    def _untile(self, buf):
        if self.world == 1:
            self._set = buf
        elif self.mode == "allgather":
            self.ctx.untile_planes_device(self.gath[buf], self.w, self.h, self.world, (self.diff, self.spec))
        elif self.rank == self.root:
            self.ctx.untile_planes_device(self.gath[buf], self.w, self.h, self.world, (self.diff, self.spec),
                                          packed=True)

    def gather(self, buf=0):
        """The exchange and the untile of buffer set `buf`, synchronously (also timed alone)."""
        if self.world > 1:
            self._exchange(buf, False)
        self._untile(buf)

    def frame(self, gb, eye, variant=0):
        self.drain()
        self.trace_local(gb, eye, variant=variant)
        self.gather()
        return self.diff, self.spec

    tune_pairs = 4        # normal-priority stream pairs tune() tries (plus one high-priority pair)

    def tune(self, gb, eye, variant=0, frames=16, gain=1.015, warm=8):
        """Times `frames` pipelined frames on one stream and as many overlapped on each of
        `tune_pairs` normal stream pairs and one high-priority pair (after `warm` untimed
        frames each: the first launches on a fresh stream pay a one-time cost), keeps the
        fastest overlap if it is `gain` times faster than one stream; returns the ms / frame.
        Which hardware queues a pair lands on matters (measured on one MI355X, 1080p: one
        normal pair 1.21 ms, another 1.11, a high-priority pair 1.12, one stream 1.17), hence
        the timing; without the warm frames the first launches on the fresh streams made
        overlap look 25 % slower.  Every rank of a group must call it (the frames exchange)."""
        t = self.torch
        if self.streams is None:
            return None
        self.auto = False                             # step() below runs the chosen mode
        main = t.cuda.current_stream(self.device)
        pairs = {"one stream": None, "two streams": self.streams}
        for i in range(1, self.tune_pairs):
            pairs[f"two streams ({i + 1})"] = [t.cuda.Stream(self.device) for _ in range(2)]
        pairs["two high-priority streams"] = [t.cuda.Stream(self.device, priority=-1) for _ in range(2)]
        ms, launch = {}, {}
        for name, pair in pairs.items():
            self.drain()
            self.overlap = pair is not None
            if pair is not None:
                self.streams = pair
            for _ in range(warm):
                self.step(gb, eye, variant=variant)
            self.drain()
            e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
            ev = [(t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)) for _ in range(frames)]
            e0.record(main)
            for i in range(frames):
                self.step(gb, eye, variant=variant, events=ev[i])
            self.drain()
            e1.record(main)
            e1.synchronize()
            ms[name] = e0.elapsed_time(e1) / frames
            launch[name] = sum(a.elapsed_time(b) for a, b in ev) / frames
        best = min((k for k in pairs if pairs[k] is not None), key=lambda k: ms[k])
        self.overlap = ms[best] * gain < ms["one stream"]
        self.streams = pairs[best]
        self.tuned = {"ms": {k: round(v, 4) for k, v in ms.items()}}
        self.tuned["chosen"] = best if self.overlap else "one stream"
        self.tuned["overlap"] = self.overlap
        # the latency paid for the throughput: a launch's start-to-end time inside each loop
        # (overlapped, a frame's trace shares the chip with its neighbours and ends later)
        self.tuned["launch_ms"] = {k: round(v, 4) for k, v in launch.items()}
        ch = self.tuned["chosen"]
        self.tuned["latency_paid_ms"] = round(launch[ch] - launch["one stream"], 4)
        return self.tuned

    def step(self, gb, eye, variant=0, events=None):
        """One frame of the pipeline; the frame's outputs are complete after the next step() or drain().
        events: (start, end) CUDA events recorded around the frame's trace on the stream it runs on."""
        if self.auto:
            self.tune(gb, eye, variant=variant)
        if not self._pipelined():
            if events:
                events[0].record()
            self.trace_local(gb, eye, variant=variant)
            if events:
                events[1].record()
            self.gather()
            return
        b = self.cur
        self.cur = (b + 1) % self.nsets
        t = self.torch
        ts = None
        if self.overlap:
            main = t.cuda.current_stream(self.device)
            saved = self.ctx.stream
            if saved != main.cuda_stream:
                raise ValueError("overlap: the context's stream (set_stream) must be the current torch stream")
            ts = self.streams[b]
            ts.wait_stream(main)        # the G-buffer, and set b's last untile
            self.ctx.set_stream(ts.cuda_stream)
        try:
            with t.cuda.stream(ts) if ts is not None else _Null():
                if events:
                    events[0].record()
                self.trace_local(gb, eye, variant=variant, buf=b)
                if events:
                    events[1].record()
                works = self._exchange(b, True) if self.world > 1 else []
        finally:
            if ts is not None:
                self.ctx.set_stream(saved)
        self._retire(lazy=True)
        self.pending = (works, b, ts)

    def _retire(self, lazy):
        """Completes the pending frame.  Several ranks: the caller's stream waits for its
        exchange and un-permutes it.  One rank with overlap and `lazy`: nothing is queued on
        the caller's stream (a wait there, every frame, would hold up whatever trace stream
        shares its hardware queue); the frame's completion event is waited for when `diff` /
        `spec` are read."""
        if self.pending is None:
            return
        works, b, ts = self.pending
        self.pending = None
        cur = self.torch.cuda.current_stream(self.device)
        for w in works:
            w.wait()                                        # current stream waits for the exchange
        self._ready = None
        if ts is not None:
            if lazy and self.world == 1:
                self._ready = self.torch.cuda.Event()
                self._ready.record(ts)
            else:
                cur.wait_stream(ts)
        self._untile(b)

    def drain(self):
        """Completes the pending frame and orders the caller's current stream after every
        frame traced so far."""
        self._retire(lazy=False)
        if self.overlap and self.streams is not None:
            cur = self.torch.cuda.current_stream(self.device)
            for st in self.streams:
                cur.wait_stream(st)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def share_comm_id(dist, rank: int, root: int = 0, get_id=None) -> bytes:
    """The vct_comm_* bootstrap for processes that already share a torch.distributed
    group: rank `root` makes the ncclUniqueId (vct_comm_get_id, or `get_id()`), every
    rank receives its 128 bytes by broadcast_object_list (works over gloo and RCCL)."""
    if rank == root:
        if get_id is None:
            from . import Context
            get_id = Context.comm_get_id
        obj = [bytes(get_id())]
    else:
        obj = [None]
    dist.broadcast_object_list(obj, src=root)
    cid = obj[0]
    if not isinstance(cid, (bytes, bytearray)) or len(cid) != 128:
        raise ValueError(f"comm id: expected 128 bytes, got {type(cid).__name__} of {len(cid) if cid else 0}")
    return bytes(cid)


class PatternContext:
    """Stand-in for a vct Context in multi-rank rehearsals without a GPU
    (bench.py --dry-run, tests): its "trace" writes each owned pixel's frame index
    (diffuse plane) and its negative (specular plane) into the rank's compact
    tiles, and its untile is the host mirror above, so an assembled frame can be
    checked exactly.  Nothing is measured with it."""

    def __init__(self, torch):
        self.torch = torch

    def trace_device(self, pos4, nrm4, alb4, width, height, eye, diffuse4, spec4, tile_rank=0, tile_world=1,
                     tile_compact=False, **_):
        t = self.torch
        fi, ci = compact_index(width, height, tile_rank, tile_world) if tile_compact else \
            (np.arange(width * height), np.arange(width * height))
        v = t.from_numpy(fi.astype(np.float32))[:, None].expand(-1, 4)
        diffuse4.view(-1, 4)[t.from_numpy(ci)] = v
        spec4.view(-1, 4)[t.from_numpy(ci)] = -v

    def untile_planes_device(self, gathered4, width, height, world, frames4, packed=False):
        g = gathered4.reshape(-1, 4).numpy()
        if packed:
            outs = untile_packed(g, width, height, world, len(frames4))
        else:
            gg = g.reshape(world, len(frames4), -1, 4)
            outs = [untile(gg[:, p], width, height, world) for p in range(len(frames4))]
        for f, o in zip(frames4, outs):
            f.copy_(self.torch.from_numpy(o))
