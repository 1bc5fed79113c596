#!/usr/bin/env python3
"""Per-rank K4 time of the N-GPU screen-tile split, measured on ONE GPU.

    python tools/rank_emul.py [--worlds 1,2,4,8] [--reps 7] [--n 256 --w 1920 --h 1080]

For each world size N and each rank r < N, times exactly the launch rank r
makes in the N-GPU bench (its interleaved 64x64 tiles, rank-compact output) and
reports the slowest rank: the K4 part of the N-GPU step (the all-gather and
the untile come on top; the gather overlaps the next frame's trace).  For N > 1 it
also reports each rank's K4 time per frame when, as in vct.multi.FrameTracer at
N > 1, consecutive frames run on two streams (`k4_ms_per_frame_overlapped_*`: the
next frame's waves fill the launch's tail).

    python tools/rank_emul.py --pmc-world N [--pmc-rank 0] [--pmc-launches 20]

only repeats rank R's launch of the N-rank split (after the context settled its
form for it), for rocprofv3 to record the per-rank PMC that bench.py's roofline
uses at N > 1 (tools/k4_profile_ranks.sh -> profiles/k4_counters.json `ranksN`).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--variant", type=lambda x: int(x, 0), default=0)
    ap.add_argument("--scene", default="atrium")
    ap.add_argument("--streams", type=int, default=2, help="trace streams of the overlapped frames (<= 3)")
    ap.add_argument("--overlap1", action="store_true", help="overlapped frames at world size 1 too (whole frames)")
    ap.add_argument("--pmc-world", type=int, default=0)
    ap.add_argument("--pmc-rank", type=int, default=0)
    ap.add_argument("--pmc-launches", type=int, default=20)
    a = ap.parse_args()
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    from vct.multi import TILE, tiles_for_rank
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)
    ctx.voxelize(*scenes.SCENES["atrium"]().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR)
    ctx.build_mips()
    dev = torch.device("cuda")
    cam = Camera()
    gb = [torch.empty((a.h, a.w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, a.w, a.h, scenes.ROUGHNESS, *gb)

    def timed(fn, min_calls=1):
        ts = []
        last, run = None, 0
        for i in range(256):                  # let the context's choice for this launch settle
            fn()
            torch.cuda.synchronize()
            f = ctx.trace_form
            run = run + 1 if (f >= 0 and f == last) else 0
            last = f
            if run >= 8 and i + 1 >= min_calls:
                break
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[len(ts) // 2]

    if a.pmc_world:
        W, r = a.pmc_world, a.pmc_rank
        maxt = tiles_for_rank(a.w, a.h, 0, W)
        buf = torch.empty((2, maxt * TILE * TILE, 4), device=dev)
        launch = lambda: ctx.trace_device(*gb, a.w, a.h, cam.position, buf[0], buf[1], tile_rank=r,  # noqa: E731
                                          tile_world=W, tile_compact=W > 1, variant=a.variant)
        for _ in range(64):
            launch()
            torch.cuda.synchronize()
            if ctx.trace_form >= 0:
                break
        for _ in range(a.pmc_launches):
            launch()
        torch.cuda.synchronize()
        print(json.dumps({"world": W, "rank": r, "form": ctx.trace_form, "launches": a.pmc_launches}))
        return
    out = {}
    # the two trace streams of the overlapped frames, made once as a rank process makes them
    # (streams made per world size land on hardware queues in turn; GPU_MAX_HW_QUEUES = 4,
    # and two trace streams sharing one queue serialise: measured 4-rank overlapped 0.29 ms
    # after one world size, 0.37-0.39 ms after two)
    streams = [torch.cuda.Stream() for _ in range(a.streams)]
    S = a.streams
    for W in [int(x) for x in a.worlds.split(",")]:
        maxt = tiles_for_rank(a.w, a.h, 0, W)
        buf = torch.empty((2, maxt * TILE * TILE, 4), device=dev)
        per = []
        ov = []
        bufs = [torch.empty((2, maxt * TILE * TILE, 4), device=dev) for _ in range(S)]
        frames = 40
        # each rank's single launch, then its overlapped frames, back to back: a rank process
        # has this one workload (the context keeps four; eight ranks' keys in turn would
        # evict each other between the two measurements and re-time inside the second)
        for r in range(W):
            # >= 72 launches on one stream first: the context counts launches as overlapped
            # until 64 after the last stream switch (the previous rank's overlapped frames)
            per.append(timed(lambda: ctx.trace_device(*gb, a.w, a.h, cam.position, buf[0], buf[1], tile_rank=r,
                                                      tile_world=W, tile_compact=W > 1, variant=a.variant),
                             min_calls=72))
            if W > 1 or a.overlap1:
                def loop():
                    # S frames in flight: frame f on stream f % S starts once frame f - S + 1 ended
                    for f in range(frames):
                        st = streams[f % S]
                        st.wait_stream(stream)
                        ctx.set_stream(st.cuda_stream)
                        b = bufs[f % S]
                        ctx.trace_device(*gb, a.w, a.h, cam.position, b[0], b[1], tile_rank=r, tile_world=W,
                                         tile_compact=True, variant=a.variant)
                        ctx.set_stream(stream.cuda_stream)
                        stream.wait_stream(streams[(f + 1) % S])
                    for st_ in streams:
                        stream.wait_stream(st_)
                ov.append(timed(loop) / frames)
        gath = torch.empty((W, 2, maxt * TILE * TILE, 4), device=dev)
        fr = (torch.empty((a.h, a.w, 4), device=dev), torch.empty((a.h, a.w, 4), device=dev))
        unt = timed(lambda: ctx.untile_planes_device(gath, a.w, a.h, W, fr)) if W > 1 else 0.0
        out[W] = {"k4_ms_max_rank": round(max(per), 4), "k4_ms_min_rank": round(min(per), 4),
                  "tiles_per_rank": maxt, "untile_ms": round(unt, 4)}
        if ov:
            out[W].update({"k4_ms_per_frame_overlapped_max_rank": round(max(ov), 4),
                           "k4_ms_per_frame_overlapped_min_rank": round(min(ov), 4)})
    base = out.get(1, {}).get("k4_ms_max_rank")
    if base:
        for W, d in out.items():
            d["k4_speedup"] = round(base / d["k4_ms_max_rank"], 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
