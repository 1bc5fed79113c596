import os, sys
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]
import numpy as np
from vct import Context, scenes
n = 256
g0, E = scenes.grid_for_unit_box(n)
ctx = Context(n, g0, E)
ctx.voxelize(*scenes.SCENES["atrium"]().arrays())
ao, nm = ctx.download_voxels()
occ = ao[..., 3] > 0
l = np.array(scenes.LIGHT_DIR, np.float64); l /= np.linalg.norm(l)
ndl = (nm[..., :3].astype(np.float64) @ l)
lit = occ & (ndl > 0)
print("occupied", int(occ.sum()), "lit", int(lit.sum()))
z, y, x = np.nonzero(lit.reshape(n, n, n)) if False else (None, None, None)
idx = np.nonzero(lit.reshape(-1))[0]
xs, ys, zs = idx % n, (idx // n) % n, idx // (n * n)
q = np.stack([xs + 0.5, ys + 0.5, zs + 0.5], 1) + nm.reshape(-1, 4)[idx, :3]
# cells to the boundary along l (upper bound of the walk)
tx = np.where(l[0] > 0, (n - q[:, 0]) / l[0], np.where(l[0] < 0, -q[:, 0] / l[0], np.inf))
ty = np.where(l[1] > 0, (n - q[:, 1]) / l[1], np.where(l[1] < 0, -q[:, 1] / l[1], np.inf))
tz = np.where(l[2] > 0, (n - q[:, 2]) / l[2], np.where(l[2] < 0, -q[:, 2] / l[2], np.inf))
t = np.minimum(np.minimum(tx, ty), tz)
cells = t * np.abs(l).sum()
print("walk upper bound: mean %.1f max %.1f total %.3g" % (cells.mean(), cells.max(), cells.sum()))
r0 = ctx.download_level(0) if False else None

# --- walk lengths (float32 DDA with the kernel's tie rule; statistics only) and the lane
# utilisation of 64-lane waves in list order against waves sorted by the walk's upper bound
f32 = np.float32
L = np.array(scenes.LIGHT_DIR, np.float32); L = L / np.float32(np.sqrt(np.float32((L * L).sum())))
qf = q.astype(f32)
v = np.floor(qf).astype(np.int64)
s_ = np.sign(L).astype(np.int64)
td = np.where(s_ != 0, f32(1) / np.abs(L), f32(np.inf)).astype(f32)
tm = np.where(s_ > 0, ((v + 1).astype(f32) - qf) * td, np.where(s_ < 0, (qf - v.astype(f32)) * td, f32(np.inf))).astype(f32)
occf = occ.reshape(-1)
alive = np.ones(len(idx), bool)
walk = np.zeros(len(idx), np.int64)
for it in range(4 * n):
    ins = np.all((v >= 0) & (v < n), 1)
    alive &= ins
    if not alive.any():
        break
    cell = v[:, 0] + n * (v[:, 1] + n * v[:, 2])
    hit = alive & occf[np.where(ins, cell, 0)]
    walk += alive
    alive &= ~hit
    tmin = tm.min(1)
    bx = tm[:, 0] == tmin
    by = ~bx & (tm[:, 1] == tmin)
    bz = ~bx & ~by
    for a, b in ((0, bx), (1, by), (2, bz)):
        v[:, a] += np.where(b, s_[a], 0)
        tm[:, a] = np.where(b, tm[:, a] + td[a], tm[:, a]).astype(f32)
print("walk cells: mean %.1f p90 %.0f max %d total %d" % (walk.mean(), np.percentile(walk, 90), walk.max(), walk.sum()))
def util(order):
    w = walk[order]
    m = (len(w) + 63) // 64 * 64
    w = np.concatenate([w, np.zeros(m - len(w), np.int64)]).reshape(-1, 64)
    return w.sum() / (64 * w.max(1)).sum(), (w.max(1)).sum()
for name, order in (("list order", np.arange(len(idx))), ("sorted by bound", np.argsort(-cells, kind="stable")),
                    ("sorted by walk (ideal)", np.argsort(-walk, kind="stable"))):
    u, tot = util(order)
    print(f"{name}: lane utilisation {u:.3f}, sum of wave maxima {tot}")
