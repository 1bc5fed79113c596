#!/usr/bin/env python3
"""Would splitting a pixel block's cones over two waves shorten the N-GPU tail?

    python tools/split_emul.py [--worlds 1,2,4,8] [--reps 7]

For rank 0's tiles at each world size: K4 with all cones (9 diffuse + spec),
diffuse-only and spec-only, and the diffuse-only and spec-only launches run
concurrently on two streams (an upper bound on what a two-wave cone split
could reach, minus the combine step).
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
    a = ap.parse_args()
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    from vct.multi import TILE, tiles_for_rank
    n, w, h = 256, 1920, 1080
    g0, E = scenes.grid_for_unit_box(n)
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    arrs = scenes.SCENES["atrium"]().arrays()
    ctxs = {}
    for name, nd, sp, st in [("all", 9, True, s0), ("diff", 9, False, s0), ("spec", 0, True, s1)]:
        c = Context(n, g0, E, n_diffuse=nd, specular=sp)
        c.set_stream(st.cuda_stream)
        c.voxelize(*arrs)
        c.inject_directional(scenes.LIGHT_DIR)
        c.build_mips()
        ctxs[name] = c
    torch.cuda.synchronize()
    dev = torch.device("cuda")
    cam = Camera()
    gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
    ctxs["all"].gbuffer_raycast_device(cam, w, h, scenes.ROUGHNESS, *gb)
    torch.cuda.synchronize()

    def timed(launch):
        ts = []
        launch()
        torch.cuda.synchronize()
        for _ in range(a.reps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e2 = torch.cuda.Event(enable_timing=True)
            e0.record(s0)
            s1.wait_event(e0)
            launch()
            e1.record(s0)
            e2.record(s1)
            torch.cuda.synchronize()
            ts.append(max(e0.elapsed_time(e1), e0.elapsed_time(e2)))
        return round(sorted(ts)[len(ts) // 2], 4)

    out = {}
    for W in [int(x) for x in a.worlds.split(",")]:
        maxt = tiles_for_rank(w, h, 0, W)
        bufs = {k: (torch.empty((maxt * TILE * TILE, 4), device=dev), torch.empty((maxt * TILE * TILE, 4), device=dev))
                for k in ctxs}

        def run(k):
            ctxs[k].trace_device(*gb, w, h, cam.position, *bufs[k], tile_rank=0, tile_world=W,
                                 tile_compact=True)
        out[W] = {"all": timed(lambda: run("all")), "diff": timed(lambda: run("diff")),
                  "spec": timed(lambda: run("spec")),
                  "diff||spec": timed(lambda: (run("diff"), run("spec")))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
