#!/usr/bin/env python3
"""What would sorting pixels into coherent waves buy K4?  (emulation, no kernel change)

    python tools/sort_emul.py [--scene atrium] [--n 256] [--w 1920 --h 1080]

K4 takes one 8x8 screen block per wave.  This tool sorts the valid G-buffer
pixels by a key (quantized normal, then the Morton code of the pixel's voxel at
a chosen level) and lays every 64 consecutive sorted pixels out as one wave of
a "virtual frame" (the kernel's own tile / block / Morton-lane map inverted), so
the unchanged kernel traces the sorted waves.  Per-pixel results do not depend
on which wave a pixel is in (every path is bit-identical), so the outputs are
compared with the screen-order trace pixel for pixel, and both are timed.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def morton3(x, y, z, bits):
    import numpy as np
    k = np.zeros_like(x, dtype=np.uint64)
    for b in range(bits):
        k |= ((x >> b) & 1).astype(np.uint64) << np.uint64(3 * b)
        k |= ((y >> b) & 1).astype(np.uint64) << np.uint64(3 * b + 1)
        k |= ((z >> b) & 1).astype(np.uint64) << np.uint64(3 * b + 2)
    return k


def virtual_xy(q, lane):
    """kernel wave q (blockIdx order within a part, WG1) and lane -> (x, y) in a frame of 32-tile rows"""
    mx = (lane & 1) | ((lane >> 1) & 2) | ((lane >> 2) & 4)
    my = ((lane >> 1) & 1) | ((lane >> 2) & 2) | ((lane >> 3) & 4)
    rb, quarter = q >> 2, q & 3
    lt, sub = rb >> 4, rb & 15
    px = (sub & 3) * 16 + (quarter & 1) * 8 + mx
    py = (sub >> 2) * 16 + (quarter >> 1) * 8 + my
    return (lt % 32) * 64 + px, (lt // 32) * 64 + py


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="atrium")
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--level", type=int, default=1, help="voxel level of the Morton key")
    ap.add_argument("--nq", type=int, default=16, help="normal quantization steps per axis")
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    import numpy as np
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    st = torch.cuda.current_stream()
    ctx.set_stream(st.cuda_stream)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR)
    ctx.build_mips()
    dev = torch.device("cuda")
    cam = Camera()
    gb = [torch.empty((a.h, a.w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, a.w, a.h, scenes.ROUGHNESS, *gb)
    pos, nrm, alb = (t.cpu().numpy().reshape(-1, 4) for t in gb)
    valid = np.flatnonzero(pos[:, 3] != 0)
    # key: quantized normal (high bits), Morton code of the voxel at `level` (low bits)
    q = np.clip(((nrm[valid, :3] + 1) * 0.5 * a.nq).astype(np.int64), 0, a.nq - 1)
    nkey = (q[:, 0] * a.nq + q[:, 1]) * a.nq + q[:, 2]
    vox = np.clip(((pos[valid, :3] - np.asarray(g0)) * (a.n / E)).astype(np.int64) >> a.level, 0,
                  (a.n >> a.level) - 1)
    bits = int(np.log2(a.n >> a.level))
    key = (nkey.astype(np.uint64) << np.uint64(3 * bits)) | morton3(vox[:, 0], vox[:, 1], vox[:, 2], bits)
    order = valid[np.argsort(key, kind="stable")]
    nw = (order.size + 63) // 64
    ntiles = (nw + 63) // 64
    W, H = 32 * 64, ((ntiles + 31) // 32) * 64
    qi = np.arange(order.size) // 64
    li = np.arange(order.size) % 64
    vx, vy = virtual_xy(qi, li)
    vidx = vy * W + vx
    vgb = []
    for src in (pos, nrm, alb):
        dst = np.zeros((H * W, 4), np.float32)
        dst[vidx] = src[order]
        vgb.append(torch.from_numpy(dst.reshape(H, W, 4)).to(dev))

    def run(g, w, h, reps):
        d, s = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
        ctx.trace_device(*g, w, h, cam.position, d, s)
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            ctx.trace_device(*g, w, h, cam.position, d, s)
            e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[len(ts) // 2], d, s

    t0, d0, s0 = run(gb, a.w, a.h, a.reps)
    t1, d1, s1 = run(vgb, W, H, a.reps)
    t0b, _, _ = run(gb, a.w, a.h, a.reps)
    same = bool(np.array_equal(d1.cpu().numpy().reshape(-1, 4)[vidx], d0.cpu().numpy().reshape(-1, 4)[order]) and
                np.array_equal(s1.cpu().numpy().reshape(-1, 4)[vidx], s0.cpu().numpy().reshape(-1, 4)[order]))
    print(json.dumps({"scene": a.scene, "screen_ms": round(min(t0, t0b), 4), "sorted_ms": round(t1, 4),
                      "valid_px": int(order.size), "sorted_waves": int(nw), "virtual_frame": [W, H],
                      "level": a.level, "nq": a.nq, "same_pixels": same}))


if __name__ == "__main__":
    main()
