#!/usr/bin/env python3
"""Row f2 timing: brute-force ray caster vs tile-binned G-buffer pass.

    python tools/gbuffer_bench.py [--tris 20000] [--w 1920 --h 1080]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=20000)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    s = scenes.random_triangles(a.tris, seed=3, size=0.08)
    g0, E = scenes.grid_for_unit_box(64)
    ctx = Context(64, g0, E)
    st = torch.cuda.current_stream()
    ctx.set_stream(st.cuda_stream)
    ctx.voxelize(*s.arrays())
    dev = torch.device("cuda")
    cam = Camera()
    out = {}
    bufs = {k: [torch.empty((a.h, a.w, 4), device=dev) for _ in range(3)] for k in ("raycast", "raster")}
    for name, fn in (("raster", ctx.gbuffer_raster_device), ("raycast", ctx.gbuffer_raycast_device)):
        fn(cam, a.w, a.h, 0.1, *bufs[name])
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn(cam, a.w, a.h, 0.1, *bufs[name])
            e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name + "_ms"] = round(sorted(ts)[len(ts) // 2], 3)
    out["identical"] = all(torch.equal(x, y) for x, y in zip(bufs["raycast"], bufs["raster"]))
    out.update(tris=a.tris, w=a.w, h=a.h)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
