#!/usr/bin/env python3
"""One bench workload's kernels, repeated for rocprofv3 (the per-line roofline records).

    python tools/pmc_workload.py --wl c3|courtyard|rand|c4|c5 [--world N] [--rank 0] [--launches 10]

Runs exactly what bench.py runs for that line -- the same scene, grid, frame, cone set,
G-buffer (the HIP raster from the reference camera; G_rand with seed 42 for `rand`) and
default variant -- on one GPU: K1 (voxelize_device) x3, K2 (inject) x10, K3 (build_mips)
x10 (the first after K1 a full build, the others relight builds), one counting K4 launch, the launches the K4 tuner needs to settle (as
bench.settle_form), then `--launches` timed K4 launches of the settled form.  With
--world N it is rank `--rank`'s own launch of the N-rank screen-tile split (compact
output), the launch bench.py's rank 0 times at N GPUs.  Prints one JSON line (the
workload's profile key, its counting-pass cone steps / texels / valid pixels, the form)
that tools/make_pmc_records.py combines with the rocprofv3 passes of the same command
(tools/pmc_all.sh).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]

# bench.py's lines: (scene, grid, width, height, diffuse cones, G-buffer)
WORKLOADS = {
    "c3": ("atrium", 256, 1920, 1080, 9, "scene"),
    "courtyard": ("courtyard", 256, 1920, 1080, 9, "scene"),
    "rand": ("atrium", 256, 1920, 1080, 9, "rand"),
    "c4": ("atrium", 512, 3840, 2160, 9, "scene"),
    "c5": ("courtyard", 512, 3840, 2160, 16, "scene"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wl", required=True, choices=sorted(WORKLOADS))
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--relight", type=int, default=10, help="K2 / K3 calls (K1: 3)")
    ap.add_argument("--variant", type=lambda v: int(v, 0), default=0)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from vct import Context, scenes
    from vct.camera import Camera
    from vct.multi import TILE, tiles_for_rank

    scene, n, w, h, nd, gbk = WORKLOADS[a.wl]
    dev = torch.device("cuda", 0)
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E, aniso=True, n_diffuse=nd, specular=True, device=0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)
    v, i, m, k = scenes.SCENES[scene]().arrays()
    dgeo = (torch.from_numpy(v).to(dev), torch.from_numpy(i.astype(np.int32)).to(dev),
            torch.from_numpy(m.astype(np.int32)).to(dev), torch.from_numpy(k).to(dev))
    for _ in range(3):
        ctx.voxelize_device(*dgeo)
    for _ in range(a.relight):
        ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    for _ in range(a.relight):
        ctx.build_mips()
    torch.cuda.synchronize()
    cam = Camera()
    eye = [float(x) for x in cam.position]
    if gbk == "scene":
        gb = tuple(torch.empty((h, w, 4), dtype=torch.float32, device=dev) for _ in range(3))
        ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)
    else:
        ao, nm = ctx.download_voxels()
        gb = tuple(torch.from_numpy(x).to(dev) for x in scenes.gbuffer_rand(ao, nm, ctx.aabb_min, ctx.extent, w, h,
                                                                             seed=42))
    W, r = a.world, a.rank
    if W > 1:
        maxt = tiles_for_rank(w, h, 0, W)
        out = torch.empty((2, maxt * TILE * TILE, 4), device=dev)
        d, sp = out[0], out[1]
        tile = dict(tile_rank=r, tile_world=W, tile_compact=True)
    else:
        d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
        tile = {}
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    ctx.trace_device(*gb, w, h, eye, d, sp, cone_steps=cnt[0:1], texel_fetches=cnt[1:2], variant=a.variant, **tile)
    torch.cuda.synchronize()
    valid = (gb[0][..., 3] != 0).reshape(-1).cpu().numpy()
    if W > 1:
        from vct.multi import compact_index
        fi, _ = compact_index(w, h, r, W)
        valid_px = int(valid[fi].sum())
    else:
        valid_px = int(valid.sum())
    form = bench.settle_form(ctx, torch, lambda: ctx.trace_device(*gb, w, h, eye, d, sp, variant=a.variant, **tile))
    for _ in range(a.launches):
        ctx.trace_device(*gb, w, h, eye, d, sp, variant=a.variant, **tile)
    torch.cuda.synchronize()
    key = bench.profile_key(n, w, h, scene, gbk, nd, True, a.variant, W)
    print(json.dumps({"key": key, "workload": a.wl, "world": W, "rank": r, "cone_steps": int(cnt[0].item()),
                      "texel_fetches": int(cnt[1].item()), "valid_px": valid_px, "form": form,
                      "form_name": bench.form_name(form), "launches": a.launches, "relight_calls": a.relight,
                      "k1_calls": 3, "occupied_voxels": None, "k3_first_build_full": True}))
    ctx.close()


if __name__ == "__main__":
    main()
