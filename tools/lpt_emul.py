#!/usr/bin/env python3
"""Longest-first dispatch of one rank's K4 launch, from a recorded duration per unit.

    python tools/lpt_emul.py [--world 8 --rank 0] [--reps 9] [--variant 0]

Settles the rank's launch (the tuner's form), records every unit's (workgroup's) wave
duration once (vct_debug_k4_sched: s_memrealtime per wave), builds a dispatch order that
keeps each unit on its XCD (blockIdx % 8) and puts the XCD's units longest first, then
times the launch in blockIdx order and in that order, alternating, and checks that the
two give the same outputs bit for bit.  An oracle for a frame-to-frame schedule: the
durations come from the same frame.
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--variant", type=lambda x: int(x, 0), default=0)
    ap.add_argument("--scene", default="atrium")
    a = ap.parse_args()
    import numpy as np
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    from vct.multi import TILE, tiles_for_rank
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR)
    ctx.build_mips()
    lib = ctx.lib
    lib.vct_debug_k4_sched.restype = C.c_int
    lib.vct_debug_k4_sched.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda")
    cam = Camera()
    gb = [torch.empty((a.h, a.w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, a.w, a.h, scenes.ROUGHNESS, *gb)
    W = a.world
    opx = tiles_for_rank(a.w, a.h, a.rank, W) * TILE * TILE if W > 1 else a.w * a.h
    var = a.variant | (0x4000000 if W == 1 and not a.variant & 0x8000 else 0)
    outs = [(torch.empty((opx, 4), device=dev), torch.empty((opx, 4), device=dev)) for _ in range(2)]

    def launch(o):
        ctx.trace_device(*gb, a.w, a.h, cam.position, *o, tile_rank=a.rank, tile_world=W, tile_compact=W > 1,
                         variant=var)

    for _ in range(256):
        launch(outs[0])
        torch.cuda.synchronize()
        if ctx.trace_form >= 0:
            break
    nunits = 1 << 20
    dur = torch.zeros(nunits, dtype=torch.int32, device=dev)
    lib.vct_debug_k4_sched(ctx.h, None, C.c_void_p(dur.data_ptr()))
    for _ in range(3):
        launch(outs[0])
    torch.cuda.synchronize()
    lib.vct_debug_k4_sched(ctx.h, None, None)
    d = dur.cpu().numpy().astype(np.int64)
    used = int(np.flatnonzero(d).max()) + 1
    d = d[:used]
    order = np.empty(used, np.int64)
    for x in range(8):                         # each XCD keeps its units, longest first
        ids = np.arange(x, used, 8)
        order[ids] = ids[np.argsort(-d[ids], kind="stable")]
    ordt = torch.from_numpy(order.astype(np.int32)).to(dev)

    def timed(with_order):
        lib.vct_debug_k4_sched(ctx.h, C.c_void_p(ordt.data_ptr()) if with_order else None, None)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        launch(outs[1 if with_order else 0])
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1)

    ts = {False: [], True: []}
    for _ in range(a.reps):
        for w in (False, True):
            ts[w].append(timed(w))
    lib.vct_debug_k4_sched(ctx.h, None, None)
    same = bool(torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]))
    med = {k: sorted(v)[len(v) // 2] for k, v in ts.items()}
    us = d / 100.0
    print(json.dumps({"world": W, "rank": a.rank, "form": ctx.trace_form, "units": used,
                      "unit_us_mean_max": [round(float(us.mean()), 1), round(float(us.max()), 1)],
                      "blockidx_order_ms": round(med[False], 4), "longest_first_ms": round(med[True], 4),
                      "bitexact": same}))


if __name__ == "__main__":
    main()
