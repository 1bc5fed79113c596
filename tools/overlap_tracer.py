"""FrameTracer's frame loop on one GPU (bench.py's timed loop without the rest of the
bench): ms per frame with and without two-stream overlap, and the same two streams
driven by hand (null stream + one pool stream, or two pool streams), to see which
stream arrangement lets consecutive K4 launches overlap.

    python tools/overlap_tracer.py [--frames 40]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--world", type=int, default=1, help="trace rank 0's tiles of this many ranks")
    a = ap.parse_args()
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    from vct.multi import FrameTracer
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    main_s = torch.cuda.current_stream()
    ctx.set_stream(main_s.cuda_stream)
    ctx.voxelize(*scenes.atrium().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ctx.build_mips()
    dev = torch.device("cuda")
    cam = Camera()
    eye = [float(x) for x in cam.position]
    gb = [torch.empty((a.h, a.w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, a.w, a.h, scenes.ROUGHNESS, *gb)
    torch.cuda.synchronize()
    print("main stream", main_s.cuda_stream, flush=True)

    def wall(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3 / a.frames

    for overlap in ((False, True, False, True) if a.world == 1 else ()):
        tr = FrameTracer(ctx, torch, None, a.w, a.h, 0, 1, dev, overlap=overlap)
        for _ in range(30):
            tr.frame(gb, eye)
        torch.cuda.synchronize()

        def loop():
            for _ in range(a.frames):
                tr.step(gb, eye)
            tr.drain()
        ms = wall(loop)
        print(f"FrameTracer overlap={overlap}: {ms:.4f} ms/frame, form {ctx.trace_form}"
              + (f", streams {[s.cuda_stream for s in tr.streams]}" if overlap else ""), flush=True)

    from vct.multi import TILE, tiles_for_rank
    W = a.world
    npx = tiles_for_rank(a.w, a.h, 0, W) * TILE * TILE if W > 1 else a.w * a.h
    kw = dict(tile_rank=0, tile_world=W, tile_compact=W > 1)
    outs = [(torch.empty((npx, 4), device=dev), torch.empty((npx, 4), device=dev)) for _ in range(2)]
    p0, p1, pm = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    for name, (sa, sb), wait_main, main_waits, mst in (
            ("null + pool", (main_s, p1), False, False, main_s),
            ("pool + pool", (p0, p1), False, False, main_s),
            ("one pool stream", (p0, p0), False, False, main_s),
            ("pool + pool, trace waits main", (p0, p1), True, False, main_s),
            ("pool + pool, main waits trace", (p0, p1), False, True, main_s),
            ("pool + pool, both (FrameTracer's order)", (p0, p1), True, True, main_s),
            ("pool + pool, both, main = pool stream", (p0, p1), True, True, pm),
            ("pool + pool, both, torch stream context", (p0, p1), True, True, "ctx"),
            ("pool + pool, both, ctx stream back to main", (p0, p1), True, True, "reset"),
            ("one pool stream, again", (p0, p0), False, False, main_s),
            ("pool + pool, again", (p0, p1), False, False, main_s)):
        mode = mst if isinstance(mst, str) else None
        mst = main_s if mode else mst

        def loop2():
            sa.wait_stream(mst)
            sb.wait_stream(mst)
            for f in range(a.frames):
                st, other = (sa, sb) if f % 2 == 0 else (sb, sa)
                if wait_main:
                    st.wait_stream(mst)
                ctx.set_stream(st.cuda_stream)
                if mode == "ctx":
                    with torch.cuda.stream(st):
                        ctx.trace_device(*gb, a.w, a.h, eye, outs[f % 2][0], outs[f % 2][1], **kw)
                else:
                    ctx.trace_device(*gb, a.w, a.h, eye, outs[f % 2][0], outs[f % 2][1], **kw)
                if mode == "reset":
                    ctx.set_stream(main_s.cuda_stream)
                if main_waits:
                    mst.wait_stream(other)
            ctx.set_stream(main_s.cuda_stream)
            mst.wait_stream(sa)
            mst.wait_stream(sb)
            main_s.wait_stream(mst)
        loop2()
        print(f"by hand, {name}: {wall(loop2):.4f} ms/frame", flush=True)

    if a.world > 1:
        return
    pm_tr = FrameTracer(ctx, torch, None, a.w, a.h, 0, 1, dev, overlap=True)
    with torch.cuda.stream(pm):
        ctx.set_stream(pm.cuda_stream)
        for _ in range(10):
            pm_tr.frame(gb, eye)

        def loop3():
            for _ in range(a.frames):
                pm_tr.step(gb, eye)
            pm_tr.drain()
        print(f"FrameTracer overlap=True, caller on a pool stream: {wall(loop3):.4f} ms/frame", flush=True)
    ctx.set_stream(main_s.cuda_stream)


if __name__ == "__main__":
    main()
