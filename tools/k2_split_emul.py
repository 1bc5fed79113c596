#!/usr/bin/env python3
"""What splitting the long K2 shadow walks over several lanes could buy (an emulation,
run on the GPU box: the voxels come from the HIP library).

Replays every lit voxel's walk (float32 DDA with the kernel's tie rule, as
tools/k2_stats.py) and records how many of its cells are entered in each of S equal
slices of its exit parameter te.  Then compares the 64-lane waves' maxima (a wave runs as
long as its longest lane; tools/k2_waves.py shows the launch span is its longest wave):
  * list order, one lane per walk (the kernel);
  * the walks whose upper bound exceeds B split into S segments (segment s also pays a
    skip of its earlier crossings, `--skip-cost` of a cell each), placed first, the
    others after them in list order.
    python tools/k2_split_emul.py [--scene atrium] [--n 256]
"""
import argparse
import json
import os
import sys

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="atrium")
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--skip-cost", type=float, default=0.25, help="cost of one skipped crossing, in cells")
    a = ap.parse_args()
    import numpy as np
    from vct import Context, scenes
    n = a.n
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    ao, nm = ctx.download_voxels()
    occ = ao[..., 3] > 0
    f32 = np.float32
    L = np.array(scenes.LIGHT_DIR, np.float32)
    L = L / np.float32(np.sqrt(np.float32((L * L).sum())))
    ndl = nm[..., 0] * L[0] + nm[..., 1] * L[1] + nm[..., 2] * L[2]
    lit = (occ & (ndl > 0)).reshape(-1)
    idx = np.nonzero(lit)[0]
    xs, ys, zs = idx % n, (idx // n) % n, idx // (n * n)
    nmf = nm.reshape(-1, 4)[idx, :3].astype(f32)
    qf = np.stack([(xs.astype(f32) + f32(0.5)) + nmf[:, 0], (ys.astype(f32) + f32(0.5)) + nmf[:, 1],
                   (zs.astype(f32) + f32(0.5)) + nmf[:, 2]], 1).astype(f32)
    v = np.floor(qf).astype(np.int64)
    s_ = np.sign(L).astype(np.int64)
    td = np.where(s_ != 0, f32(1) / np.abs(L), f32(np.inf)).astype(f32)
    tm = np.where(s_ > 0, ((v + 1).astype(f32) - qf) * td,
                  np.where(s_ < 0, (qf - v.astype(f32)) * td, f32(np.inf))).astype(f32)
    Nf = f32(n)
    te = np.full(len(idx), np.inf, f32)
    for ax in range(3):
        if s_[ax]:
            te = np.minimum(te, ((Nf - qf[:, ax]) if s_[ax] > 0 else qf[:, ax]) * td[ax]).astype(f32)
    bound = te * f32(np.abs(L).sum())
    SMAX = 8
    seg_cells = np.zeros((len(idx), SMAX), np.int64)     # cells entered per 1/SMAX slice of te
    occf = occ.reshape(-1)
    alive = np.ones(len(idx), bool)
    entry = np.zeros(len(idx), f32)
    for _ in range(4 * n):
        ins = np.all((v >= 0) & (v < n), 1)
        alive &= ins
        if not alive.any():
            break
        cell = v[:, 0] + n * (v[:, 1] + n * v[:, 2])
        hit = alive & occf[np.where(ins, cell, 0)]
        sl = np.clip(np.floor(entry / te * SMAX).astype(np.int64), 0, SMAX - 1)
        np.add.at(seg_cells, (np.flatnonzero(alive), sl[alive]), 1)
        alive &= ~hit
        tmin = tm.min(1)
        entry = tmin
        bx = tm[:, 0] == tmin
        by = ~bx & (tm[:, 1] == tmin)
        bz = ~bx & ~by
        for ax, b in ((0, bx), (1, by), (2, bz)):
            v[:, ax] += np.where(b, s_[ax], 0)
            tm[:, ax] = np.where(b, tm[:, ax] + td[ax], tm[:, ax]).astype(f32)
    walk = seg_cells.sum(1)

    def waves(cost):
        m = (len(cost) + 63) // 64 * 64
        w = np.concatenate([cost, np.zeros(m - len(cost))]).reshape(-1, 64).max(1)
        return {"waves": int(len(w)), "max": round(float(w.max()), 1),
                "p99_p90_p50": [round(float(np.percentile(w, q)), 1) for q in (99, 90, 50)],
                "sum": round(float(w.sum()), 1)}

    out = {"scene": a.scene, "n": n, "lit": int(len(idx)),
           "walk_mean_p90_max": [round(float(walk.mean()), 1), float(np.percentile(walk, 90)), int(walk.max())],
           "list_order": waves(walk.astype(float))}
    for S in (2, 4):
        for frac in (0.05, 0.1, 0.2):
            B = float(np.percentile(bound, 100 * (1 - frac)))
            long_ = bound > B
            per = SMAX // S
            segs = []
            for s in range(S):
                c = seg_cells[long_, s * per:(s + 1) * per].sum(1).astype(float)
                skipped = seg_cells[long_, :s * per].sum(1) + 0.0   # the crossings before the segment
                segs.append(c + a.skip_cost * skipped + (1.0 if s else 0.0))
            seg = np.stack(segs, 1).reshape(-1)
            cost = np.concatenate([seg, walk[~long_].astype(float)])
            out[f"S{S}_top{int(frac * 100)}pct"] = waves(cost)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
