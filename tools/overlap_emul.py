"""Frame overlap on one GPU: consecutive K4 frames on one stream (each waits for the one
before) vs alternating two streams (frame f+1's waves fill the slots frame f's tail leaves
idle), for the full frame and for rank 0's launch of an N-rank split.  Outputs of the two
buffer sets are checked bit-equal to the single-stream frame.

    python tools/overlap_emul.py [--worlds 1,2,4,8] [--frames 40]
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
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--scene", default="atrium")
    ap.add_argument("--variant", type=lambda v: int(v, 0), default=0,
                    help="trace variant (0x1000000 union form, 0x2000000 occupancy form)")
    a = ap.parse_args()
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    from vct.multi import TILE, tiles_for_rank
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    ctx.set_stream(s0.cuda_stream)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR)
    ctx.build_mips()
    dev = torch.device("cuda")
    cam = Camera()
    gb = [torch.empty((a.h, a.w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, a.w, a.h, scenes.ROUGHNESS, *gb)
    torch.cuda.synchronize()
    out = {}
    for W in [int(x) for x in a.worlds.split(",")]:
        npx = tiles_for_rank(a.w, a.h, 0, W) * TILE * TILE if W > 1 else a.w * a.h
        bufs = [(torch.empty((npx, 4), device=dev), torch.empty((npx, 4), device=dev)) for _ in range(2)]
        kw = dict(tile_rank=0, tile_world=W, tile_compact=W > 1, variant=a.variant)

        def launch(b, stream):
            ctx.set_stream(stream.cuda_stream)
            ctx.trace_device(*gb, a.w, a.h, cam.position, bufs[b][0], bufs[b][1], **kw)

        for _ in range(40):                     # settle the tuner on s0
            launch(0, s0)
            torch.cuda.synchronize()
        ref = (bufs[0][0].clone(), bufs[0][1].clone())
        res = {}
        for mode in ("one stream", "two streams"):
            ev = [torch.cuda.Event() for _ in range(a.frames)]
            torch.cuda.synchronize()
            t0 = torch.cuda.Event(enable_timing=True)
            t1 = torch.cuda.Event(enable_timing=True)
            t0.record(s0)
            s1.wait_stream(s0)
            for f in range(a.frames):
                st = s0 if (mode == "one stream" or f % 2 == 0) else s1
                b = f % 2
                if f >= 2:                      # the buffer set's previous frame is done (read by an exchange)
                    st.wait_event(ev[f - 2])
                launch(b, st)
                ev[f].record(st)
            s0.wait_stream(s1)
            t1.record(s0)
            torch.cuda.synchronize()
            ok = all(torch.equal(bufs[b][0], ref[0]) and torch.equal(bufs[b][1], ref[1]) for b in range(2))
            res[mode] = {"ms_per_frame": round(t0.elapsed_time(t1) / a.frames, 4), "bitexact": ok}
        ctx.set_stream(s0.cuda_stream)
        res["gain"] = round(res["one stream"]["ms_per_frame"] / res["two streams"]["ms_per_frame"], 3)
        out[W] = res
        print(W, json.dumps(res), flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
