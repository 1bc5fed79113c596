#!/usr/bin/env python3
"""Level-0 footprint statistics of K4's waves (CPU, no GPU): how the 64 lanes of an
8x8 pixel wave spread at the level-0 samples of each cone, which staging shapes would
hold them, and how many of those samples are exactly zero (empty space).

    python tools/l0_emul.py [--n 256 --w 1920 --h 1080 --scene atrium]

Uses the CPU backend of include/vct.h (the oracle; test infrastructure) for K1-K3 and
the G-buffer raster, then replays the spec's step recurrence (vct_spec.h) per lane in
float64 (close enough for footprint statistics; the kernels' float32 positions differ
by ulps).  Steps with l0 = 0 only: the diffuse cones' first two steps (t = 1, 1.58) and
the specular cone's steps up to D = 2.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd"), os.path.join(REPO, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--scene", default="atrium")
    a = ap.parse_args()
    from oracle import oracle as O
    from vct import Context, _lib, scenes
    from vct.camera import Camera
    from spec_ref import CONES9
    O.build()
    lib = _lib.bind(C.CDLL(O.CPU_BACKEND))
    n, w, h = a.n, a.w, a.h
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E, lib=lib)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ctx.build_mips()
    cam = Camera()
    gb = [np.zeros((h, w, 4), np.float32) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *[b.ctypes.data for b in gb])
    r0 = ctx.download_level(0).reshape(n, n, n, 4)       # [z][y][x]
    nz = np.any(r0 != 0, axis=-1)
    pos, nrm, alb = gb
    inv_h = n / E
    o = (pos[..., :3].astype(np.float64) - np.array(g0)) * inv_h + nrm[..., :3]
    valid = pos[..., 3] != 0
    # 8x8 waves
    H8, W8 = h // 8, w // 8
    def waves(x):
        return x[:H8 * 8, :W8 * 8].reshape(H8, 8, W8, 8, *x.shape[2:]).swapaxes(1, 2).reshape(H8 * W8, 64, *x.shape[2:])
    ow, vw, nw = waves(o), waves(valid), waves(nrm[..., :3].astype(np.float64))
    keep = vw.any(axis=1)
    ow, vw, nw = ow[keep], vw[keep], nw[keep]
    pw = waves(pos[..., :3].astype(np.float64))[keep]
    print(f"waves with valid pixels: {len(ow)}")

    def frame(nv):
        nx, ny, nz_ = nv[..., 0], nv[..., 1], nv[..., 2]
        sgn = np.where(nz_ >= 0, 1.0, -1.0)
        ka = -1.0 / (sgn + nz_)
        kb = nx * ny * ka
        T = np.stack([1.0 + sgn * nx * nx * ka, sgn * kb, -sgn * nx], -1)
        B = np.stack([kb, sgn + ny * ny * ka, -ny], -1)
        return T, B

    def stats(q, name):
        """q: [waves, 64, 3] sample positions of one (cone, step); valid lanes vw"""
        c = np.floor(q - 0.5).astype(np.int64)
        big = np.where(vw[..., None], c, 1 << 40)
        small = np.where(vw[..., None], c, -(1 << 40))
        lo, hi = big.min(1), small.max(1)
        span = hi - lo + 2                                    # corner extent per axis (texels)
        # zero: all 8 corners of every valid lane are empty (texel outside = 0)
        zero_lane = np.ones(c.shape[:2], bool)
        for dz in (0, 1):
            for dy in (0, 1):
                for dx in (0, 1):
                    x, y, z = c[..., 0] + dx, c[..., 1] + dy, c[..., 2] + dz
                    ins = (x >= 0) & (x < n) & (y >= 0) & (y < n) & (z >= 0) & (z < n)
                    occ = np.zeros(x.shape, bool)
                    occ[ins] = nz[z[ins], y[ins], x[ins]]
                    zero_lane &= ~occ
        zero_wave = np.all(zero_lane | ~vw, axis=1)
        return span, zero_lane, zero_wave

    out = {}
    # diffuse: level-0 steps
    tau = 0.577350259
    ts = []
    t = 1.0
    while True:
        D = max(1.0, 2 * tau * t)
        if np.log2(D) >= 1:
            break
        ts.append(t)
        t += 0.5 * D
    T, B = frame(nw)
    spans, zl, zw = [], [], []
    for cn, ct, cb, _ in CONES9:
        d = cn * nw + ct * T + cb * B
        for t in ts:
            s, zlane, zwave = stats(ow + d * t, "diff")
            spans.append(s)
            zl.append(zlane[vw].mean())
            zw.append(zwave.mean())
    sp = np.stack(spans)                                       # [cone-steps, waves, 3]
    fit4 = np.all(sp <= 4, -1)
    smax = np.sort(sp, -1)                                     # per sample sorted spans
    out["diffuse_l0"] = {"steps": ts, "samples": int(sp.shape[0] * sp.shape[1]), "fit_4x4x4": float(fit4.mean()),
                         "fit_8x8x2_any_orientation": float(np.all(smax <= [2, 8, 8], -1).mean()),
                         "fit_6x6x6": float(np.all(sp <= 6, -1).mean()),
                         "fit_8x8x4_any": float(np.all(smax <= [4, 8, 8], -1).mean()),
                         "lane_zero_frac": float(np.mean(zl)), "wave_zero_frac": float(np.mean(zw))}
    # union region of all 9 cones' level-0 steps per wave
    reg = sp.max(0)   # not exact union (spans of different samples are not aligned); compute properly below
    q_all = []
    for cn, ct, cb, _ in CONES9:
        d = cn * nw + ct * T + cb * B
        for t in ts:
            q_all.append(np.floor(ow + d * t - 0.5).astype(np.int64))
    qa = np.stack(q_all, 1)                                    # [waves, cone-steps, 64, 3]
    vv = np.broadcast_to(vw[:, None, :, None], qa.shape)
    lo = np.where(vv, qa, 1 << 40).min((1, 2))
    hi = np.where(vv, qa, -(1 << 40)).max((1, 2))
    ext = hi - lo + 2
    vol = ext.prod(-1)
    out["diffuse_l0_union_region"] = {"texels_p50": float(np.percentile(vol, 50)), "p75": float(np.percentile(vol, 75)),
                                      "p90": float(np.percentile(vol, 90)),
                                      "frac_le_256": float((vol <= 256).mean()), "frac_le_384": float((vol <= 384).mean()),
                                      "ext_p50": np.percentile(ext, 50, axis=0).tolist()}
    # specular: r = reflect(-v, n), tau = roughness 0.1
    eye = np.array(cam.position, np.float64)
    vvec = eye - pw
    vvec /= np.linalg.norm(vvec, axis=-1, keepdims=True)
    ndv = (nw * vvec).sum(-1, keepdims=True)
    r = 2 * ndv * nw - vvec
    tau = 0.1
    ts = []
    t = 1.0
    while True:
        D = max(1.0, 2 * tau * t)
        if np.log2(D) >= 1:
            break
        ts.append(t)
        t += 0.5 * D
    spans, zl, zw, qs = [], [], [], []
    for t in ts:
        q = ow + r * t
        s, zlane, zwave = stats(q, "spec")
        spans.append(s)
        zl.append(zlane[vw].mean())
        zw.append(zwave.mean())
        qs.append(np.floor(q - 0.5).astype(np.int64))
    sp = np.stack(spans)
    smax = np.sort(sp, -1)
    out["spec_l0"] = {"steps": len(ts), "fit_4x4x4": float(np.all(sp <= 4, -1).mean()),
                      "fit_8x8x2_any": float(np.all(smax <= [2, 8, 8], -1).mean()),
                      "fit_6x6x6": float(np.all(sp <= 6, -1).mean()),
                      "lane_zero_frac": float(np.mean(zl)), "wave_zero_frac": float(np.mean(zw)),
                      "span_p50_per_step": [np.percentile(s, 50, axis=0).tolist() for s in spans[:4]]}
    qa = np.stack(qs, 1)
    vv = np.broadcast_to(vw[:, None, :, None], qa.shape)
    lo = np.where(vv, qa, 1 << 40).min((1, 2))
    hi = np.where(vv, qa, -(1 << 40)).max((1, 2))
    ext = hi - lo + 2
    vol = ext.prod(-1)
    out["spec_l0_union_region"] = {"texels_p50": float(np.percentile(vol, 50)), "p75": float(np.percentile(vol, 75)),
                                   "p90": float(np.percentile(vol, 90)),
                                   "frac_le_256": float((vol <= 256).mean()), "frac_le_384": float((vol <= 384).mean())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
