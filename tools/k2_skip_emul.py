#!/usr/bin/env python3
"""Empty-coarse-brick jumps in the K2 shadow walk, emulated (run on the GPU box: the
voxels come from the HIP library).

In a coarse brick (edge 2^cs) with no occupied voxel the walk can jump to the brick's exit
exactly: per axis, the crossings that stay inside the brick are that axis's own repeated
sum t_k+1 = t_k + td; the exit is the first (t, axis) of the three axes' leaving crossings
(ties x < y < z, the walk's own rule); the other axes take their crossings ordered before it.
The replay checks that every jumping walk ends in the same state and result as the
cell-by-cell walk, then compares the waves' maxima of slots (a slot = one cell step or one
brick jump; a jump slot costs `--jump-cost` step slots in a branch-free batch where every
slot may be either).
    python tools/k2_skip_emul.py [--scene atrium] [--n 256]
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
    ap.add_argument("--jump-cost", type=float, default=1.7)
    a = ap.parse_args()
    import numpy as np
    from vct import Context, scenes
    n = a.n
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    ao, nm = ctx.download_voxels()
    occ = (ao[..., 3] > 0).reshape(n, n, n)                       # [z][y][x]
    cs = 0
    while (n >> cs) > 64:
        cs += 1
    e = 1 << cs
    cn = n >> cs
    coarse = occ.reshape(cn, e, cn, e, cn, e).any(axis=(1, 3, 5))  # [bz][by][bx]
    f32 = np.float32
    L = np.array(scenes.LIGHT_DIR, np.float32)
    L = L / np.float32(np.sqrt(np.float32((L * L).sum())))
    ndl = nm[..., 0] * L[0] + nm[..., 1] * L[1] + nm[..., 2] * L[2]
    lit = ((ao[..., 3] > 0) & (ndl > 0)).reshape(-1)
    idx = np.nonzero(lit)[0]
    xs, ys, zs = idx % n, (idx // n) % n, idx // (n * n)
    nmf = nm.reshape(-1, 4)[idx, :3].astype(f32)
    qf = np.stack([(xs.astype(f32) + f32(0.5)) + nmf[:, 0], (ys.astype(f32) + f32(0.5)) + nmf[:, 1],
                   (zs.astype(f32) + f32(0.5)) + nmf[:, 2]], 1).astype(f32)
    s_ = np.sign(L).astype(np.int64)
    td = np.where(s_ != 0, f32(1) / np.abs(L), f32(np.inf)).astype(f32)
    v0 = np.floor(qf).astype(np.int64)
    tm0 = np.where(s_ > 0, ((v0 + 1).astype(f32) - qf) * td,
                   np.where(s_ < 0, (qf - v0.astype(f32)) * td, f32(np.inf))).astype(f32)
    occf = occ.reshape(-1)
    W = len(idx)

    def walk(jump):
        v, tm = v0.copy(), tm0.copy()
        alive = np.ones(W, bool)
        vis = np.ones(W, bool)
        slots = np.zeros(W, np.int64)
        jumps = np.zeros(W, np.int64)
        acts = []                                             # per slot: 0 done, 1 step, 2 jump
        for _ in range(4 * n):
            ins = np.all((v >= 0) & (v < n), 1)
            alive &= ins
            if not alive.any():
                break
            cell = np.where(ins, v[:, 0] + n * (v[:, 1] + n * v[:, 2]), 0)
            hit = alive & occf[cell]
            vis &= ~hit
            alive &= ~hit
            slots += alive
            vc = np.clip(v, 0, n - 1) >> cs
            empty = ~coarse[vc[:, 2], vc[:, 1], vc[:, 0]] & alive if jump else np.zeros(W, bool)
            acts.append((alive.astype(np.uint8) + empty.astype(np.uint8)))
            # one crossing (the walk's rule)
            tmin = tm.min(1)
            bx = tm[:, 0] == tmin
            by = ~bx & (tm[:, 1] == tmin)
            bz = ~bx & ~by
            nv, ntm = v.copy(), tm.copy()
            for ax, b in ((0, bx), (1, by), (2, bz)):
                nv[:, ax] += np.where(b, s_[ax], 0)
                ntm[:, ax] = np.where(b, tm[:, ax] + td[ax], tm[:, ax]).astype(f32)
            if jump and empty.any():
                # per axis: crossings to leave the brick (k), their t values t_0..t_{k-1}
                k = np.where(s_ > 0, (v | (e - 1)) - v + 1, np.where(s_ < 0, v - (v & ~(e - 1)) + 1, 1 << 30))
                ts = [tm.copy()]
                for j in range(1, e):
                    ts.append((ts[-1] + td).astype(f32))
                ts = np.stack(ts, 2)                                   # [W][3][e]
                kk = np.clip(k, 1, e)
                tex = np.take_along_axis(ts, (kk - 1)[:, :, None], 2)[:, :, 0]   # t of the leaving crossing
                tex = np.where(s_ != 0, tex, f32(np.inf)).astype(f32)
                # exit axis: min t, ties x < y < z
                ex = np.argmin(tex, 1)
                te = tex[np.arange(W), ex]
                jv, jtm = v.copy(), tm.copy()
                for ax in range(3):
                    if s_[ax] == 0:
                        continue
                    # crossings of this axis ordered before the exit event: t < te, or t == te and ax < ex
                    before = (ts[:, ax, :] < te[:, None]) | ((ts[:, ax, :] == te[:, None]) & (ax < ex)[:, None])
                    before &= np.arange(e)[None, :] < kk[:, ax:ax + 1]
                    cnt = before.sum(1) + (ex == ax)                   # the exit crossing itself
                    jv[:, ax] = v[:, ax] + s_[ax] * cnt
                    t_after = ts[:, ax, :]
                    # tm after cnt crossings: t_cnt (cnt <= e - 1 from ts, cnt == e one more add)
                    last = np.take_along_axis(t_after, np.clip(cnt, 0, e - 1)[:, None], 1)[:, 0]
                    jtm[:, ax] = np.where(cnt >= e, (t_after[:, e - 1] + td[ax]).astype(f32), last)
                nv = np.where(empty[:, None], jv, nv)
                ntm = np.where(empty[:, None], jtm, ntm).astype(f32)
                jumps += empty
            v, tm = nv, ntm
        return vis, slots, jumps, np.stack(acts, 1) if acts else np.zeros((W, 0), np.uint8)

    vis0, slots0, _, _ = walk(False)
    vis1, slots1, jumps1, act = walk(True)
    cost0 = slots0.astype(float)
    cost1 = (slots1 - jumps1) + a.jump_cost * jumps1 if False else slots1 * a.jump_cost

    def waves(cost):
        m = (len(cost) + 63) // 64 * 64
        w = np.concatenate([cost, np.zeros(m - len(cost))]).reshape(-1, 64).max(1)
        return {"max": round(float(w.max()), 1), "p99_p90_p50": [round(float(np.percentile(w, q)), 1) for q in (99, 90, 50)],
                "sum": round(float(w.sum()), 1)}

    # divergent branch per slot: a wave pays a step if any lane steps and a jump if any jumps
    m = (W + 63) // 64 * 64
    actp = np.concatenate([act, np.zeros((m - W, act.shape[1]), np.uint8)]).reshape(-1, 64, act.shape[1])
    any_step = (actp == 1).any(1)
    any_jump = (actp == 2).any(1)
    branchy = {}
    for J in (1.8, 2.6):
        c = (any_step.sum(1) + J * any_jump.sum(1)).astype(float)
        branchy[str(J)] = {"max": round(float(c.max()), 1), "p99_p90_p50": [round(float(np.percentile(c, q)), 1) for q in (99, 90, 50)],
                           "sum": round(float(c.sum()), 1)}
    print(json.dumps({"scene": a.scene, "n": n, "cs": cs, "lit": W, "branchy_wave_cost_by_jump_cost": branchy,
                      "same_result": bool(np.array_equal(vis0, vis1)),
                      "slots_mean_max": [[round(float(slots0.mean()), 1), int(slots0.max())],
                                         [round(float(slots1.mean()), 1), int(slots1.max())]],
                      "jump_fraction_of_slots": round(float(jumps1.sum() / max(1, slots1.sum())), 3),
                      "cell_steps_waves": waves(cost0),
                      f"jump_waves_at_cost_{a.jump_cost}": waves(cost1)}))


if __name__ == "__main__":
    main()
