#!/usr/bin/env python3
"""K4's brick cache replayed on the CPU (no GPU): how each (wave, step, level) sample of
the metric frame is served -- cache hit, empty space, 4^3 staging, 6^3 staging (the
policy under study), or per-lane gathers -- for a random sample of 8x8 waves.

    python tools/brick_emul.py [--waves 2000] [--wide 0|1] [--scene atrium]

Same setup as tools/zero_emul.py (CPU backend of include/vct.h, float64 restatement of
the step recurrence).  The cache follows step_bricks (vct_trace.hip): entry A holds
level l0, entry B level l0 + 1, B moves into A when the level advances; a miss of A
first tests for empty space (approximated here by the exact footprint test, which the
kernel's dilated maps only over-approximate), then stages if the active lanes fit a
brick (origin = min on axes the cone moves toward +, max - (size - 2) toward -), else
gathers.  Level B has no empty-space test.  --wide 1: a miss that does not fit 4^3 but
fits 6^3 stages 6^3 in iso / combined-face (dir_uniform) mode.
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
    ap.add_argument("--waves", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--wide", type=int, default=1)
    ap.add_argument("--nzfit", type=int, default=0,
                    help="1: a level-A miss fits / clusters only the lanes whose footprint may be nonzero")
    ap.add_argument("--multi", type=int, default=0,
                    help="K >= 2: a miss that fits no single 4^3 brick is covered by up to K "
                         "4^3 bricks (greedy lane clusters) in iso / combined-face mode")
    a = ap.parse_args()
    from oracle import oracle as O
    from vct import Context, _lib, scenes
    from vct.camera import Camera
    from spec_ref import CONES9
    O.build()
    lib = _lib.bind(C.CDLL(O.CPU_BACKEND))
    n, w, h = a.n, a.w, a.h
    L = int(np.log2(n))
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E, lib=lib)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ctx.build_mips()
    cam = Camera()
    gb = [np.zeros((h, w, 4), np.float32) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *[b.ctypes.data for b in gb])
    nzp, pyr = [], []                          # per level: nonzero texel (any face) / faces, padded by one
    for l in range(L + 1):
        nl, F = ctx.level_dims(l)[0], ctx.level_dims(l)[1]
        pad = np.zeros((F, nl + 2, nl + 2, nl + 2, 4), np.float32)
        for f in range(F):
            pad[f, 1:-1, 1:-1, 1:-1] = ctx.download_level(l, f).reshape(nl, nl, nl, 4)
        pyr.append(pad)
        nzp.append(np.any(pad != 0, axis=(0, 4)))
    FACES = ((0, 1), (2, 3), (4, 5))

    def sample_alpha(l, q, d):
        c = q * 2.0 ** -l - 0.5
        fl = np.floor(c)
        f = c - fl
        i = np.clip(fl.astype(np.int64) + 1, 0, pyr[l].shape[1] - 2)
        acc = np.zeros(q.shape[:2])
        wgt = d * d
        for dz in (0, 1):
            for dy in (0, 1):
                for dx in (0, 1):
                    wc = (f[..., 0] if dx else 1 - f[..., 0]) * (f[..., 1] if dy else 1 - f[..., 1]) * \
                         (f[..., 2] if dz else 1 - f[..., 2])
                    z, y, x = i[..., 2] + dz, i[..., 1] + dy, i[..., 0] + dx
                    if l == 0:
                        v = pyr[0][0, z, y, x, 3]
                    else:
                        v = 0
                        for ax in range(3):
                            fid = np.where(d[..., ax] >= 0, FACES[ax][0], FACES[ax][1])
                            v = v + wgt[..., ax] * pyr[l][fid, z, y, x, 3]
                    acc += wc * v
        return acc
    pos, nrm, alb = gb
    inv_h = n / E
    H8, W8 = h // 8, w // 8
    rng = np.random.default_rng(a.seed)

    def waves(x):
        return x[:H8 * 8, :W8 * 8].reshape(H8, 8, W8, 8, *x.shape[2:]).swapaxes(1, 2).reshape(H8 * W8, 64, *x.shape[2:])
    vw_all = waves(pos[..., 3] != 0)
    cand = np.nonzero(vw_all.any(1))[0]
    sel = rng.choice(cand, size=min(a.waves, len(cand)), replace=False)
    P = waves(pos[..., :3].astype(np.float64))[sel]
    N = waves(nrm[..., :3].astype(np.float64))[sel]
    V = vw_all[sel]
    Wn = len(sel)
    o = (P - np.array(g0)) * inv_h + N
    eye = np.array(cam.position, np.float64)
    BIG = 1 << 40

    def frame(nv):
        nx, ny, nz_ = nv[..., 0], nv[..., 1], nv[..., 2]
        sgn = np.where(nz_ >= 0, 1.0, -1.0)
        ka = -1.0 / (sgn + nz_)
        kb = nx * ny * ka
        return (np.stack([1.0 + sgn * nx * nx * ka, sgn * kb, -sgn * nx], -1), np.stack([kb, sgn + ny * ny * ka, -ny], -1))

    stats = {}

    def cover_bricks(c, alive, negax, sel, K, dkey=None):
        """bricks of the greedy cover (K + 1: none within K) per wave of sel: take the first
        remaining lane f, the lanes within 2 of it on every axis, their brick origin (min,
        or max - 2 toward -axis), the lanes that fit it; repeat on the rest"""
        out = np.zeros(Wn, np.int64)
        for wv in np.nonzero(sel)[0]:
            rem = alive[wv].copy()
            cw = c[wv]
            k = 0
            while rem.any() and k <= K:
                f = np.argmax(rem)
                near = rem & np.all(np.abs(cw - cw[f]) <= 2, -1)
                if dkey is not None:                 # the cluster also shares one direction (comb mode)
                    near &= np.all(dkey[wv] == dkey[wv, f], -1)
                lo_, hi_ = cw[near].min(0), cw[near].max(0)
                org = np.where(negax[wv], hi_ - 2, lo_)
                fit = near & np.all((cw >= org) & (cw <= org + 2), -1)
                rem &= ~fit
                k += 1
            out[wv] = k if not rem.any() else K + 1
        return out

    def bump(key, m):
        stats[key] = stats.get(key, 0) + int(m.sum())

    def march(kind, d, tau):
        d32 = d.astype(np.float32)
        vd = np.where(V[..., None], d32 * d32, np.nan)
        uni = np.all((vd == vd[np.arange(Wn), V.argmax(1)][:, None]) | ~V[..., None], (1, 2))
        sgnf = np.where(V[..., None], np.sign(np.where(d >= 0, 1, -1)), 0)
        nfaces = (np.any(sgnf > 0, 1) | False).sum(-1) + np.any(sgnf < 0, 1).sum(-1)
        uni &= nfaces == 3
        negax = np.all((d < 0) | ~V[..., None], 1)
        dkey = np.concatenate([(d32 * d32).view(np.uint32), (d32 < 0)], -1)             # [W, 3] the cone moves toward -axis
        alpha = np.zeros(V.shape)
        alive = V.copy()
        # cache: level, origin [W,3], size (4 or 6) per entry
        A = [np.full(Wn, -1), np.zeros((Wn, 3), np.int64), np.full(Wn, 4)]
        B = [np.full(Wn, -1), np.zeros((Wn, 3), np.int64), np.full(Wn, 4)]
        t, tmax = 1.0, n * np.sqrt(3)
        while True:
            q = o + d * t
            alive &= np.all((q >= 0) & (q <= n), -1) & (alpha < 0.95) & (t <= tmax)
            wa = alive.any(1)
            if not wa.any():
                break
            D = max(1.0, 2 * tau * t)
            m = min(np.log2(D), L)
            l0 = int(np.floor(m))
            fr = m - l0
            adv = (A[0] != l0) & (B[0] == l0)
            for i in range(3):
                A[i] = np.where(adv if i != 1 else adv[:, None], B[i], A[i])
            B[0] = np.where(adv, -1, B[0])
            for lvl, ent, isA in ((l0, A, True), (l0 + 1, B, False)):
                if not isA and not (fr > 0 and l0 < L):
                    continue
                lk = f"{kind} {'A' if isA else 'B'}"
                c = np.floor(q * 2.0 ** -lvl - 0.5).astype(np.int64)
                lo = np.where(alive[..., None], c, BIG).min(1)
                hi = np.where(alive[..., None], c, -BIG).max(1)
                span = hi - lo
                ext = ent[2][:, None] - 2
                hit = wa & (ent[0] == lvl) & np.all((lo >= ent[1]) & (hi <= ent[1] + ext), -1)
                miss = wa & ~hit
                bump(lk + " hit", hit)
                # footprint zero per lane
                zl = np.ones(V.shape, bool)
                ci = np.clip(c + 1, 0, nzp[lvl].shape[0] - 2)
                for dz in (0, 1):
                    for dy in (0, 1):
                        for dx in (0, 1):
                            zl &= ~nzp[lvl][ci[..., 2] + dz, ci[..., 1] + dy, ci[..., 0] + dx]
                empty = miss & np.all(zl | ~alive, 1) if isA else np.zeros(Wn, bool)
                bump(lk + " empty", empty)
                miss &= ~empty
                faces_ok = (lvl == 0) | uni | (nfaces <= 4)
                fitl = alive & ~zl if (isA and a.nzfit) else alive       # lanes that must fit
                lo = np.where(fitl[..., None], c, BIG).min(1)
                hi = np.where(fitl[..., None], c, -BIG).max(1)
                span = hi - lo
                wide_ok = (lvl == 0) | uni
                f4 = miss & faces_ok & np.all(span <= 2, -1)
                f6 = miss & ~f4 & wide_ok & np.all(span <= 4, -1) & bool(a.wide)
                g = miss & ~f4 & ~f6
                if a.multi >= 2:
                    # level 0 / dir_uniform waves: any lane cluster; else clusters of one direction
                    kb = np.where(wide_ok, cover_bricks(c, fitl, negax, g & wide_ok, a.multi),
                                  cover_bricks(c, fitl, negax, g & ~wide_ok, a.multi, dkey)
                                  if lvl > 0 else a.multi + 1)
                    for k_ in range(2, a.multi + 1):
                        bump(lk + f" stage4x{k_}", kb == k_)
                    g &= ~((kb >= 2) & (kb <= a.multi))
                bump(lk + " stage4", f4)
                bump(lk + " stage6", f6)
                bump(lk + " gather", g)
                bump(lk + " gather_lanes", g[:, None] & alive)
                bump(lk + " gather_lanes_aniso", g[:, None] & alive & (lvl > 0))
                for fm, sz in ((f4, 4), (f6, 6)):
                    org = np.where(negax, hi - (sz - 2), lo)
                    ent[0] = np.where(fm, lvl, ent[0])
                    ent[1] = np.where(fm[:, None], org, ent[1])
                    ent[2] = np.where(fm, sz, ent[2])
            sa = sample_alpha(l0, q, d)
            if fr > 0 and l0 < L:
                sa = (1 - fr) * sa + fr * sample_alpha(l0 + 1, q, d)
            alpha = np.where(alive, alpha + (1 - alpha) * sa, alpha)
            t = t + 0.5 * D

    T, Bv = frame(N)
    for cn, ct, cb, _ in CONES9:
        march("diffuse", cn * N + ct * T + cb * Bv, 0.577350259)
    vv = eye - P
    vv /= np.linalg.norm(vv, axis=-1, keepdims=True)
    r = 2 * (N * vv).sum(-1, keepdims=True) * N - vv
    march("spec", r, float(scenes.ROUGHNESS))
    print(json.dumps({k: v for k, v in sorted(stats.items())}, indent=1))


if __name__ == "__main__":
    main()
