"""Second, independent restatement of SURVEY.md Appendix A in numpy / pure Python
(TEST INFRASTRUCTURE; small cases only).

It exists to pin the C oracle (oracle/vct_oracle.c): the reference repository
has no implementation of this path to compare against, so the
oracle is checked bit for bit against this file on small inputs, and both are
checked against closed-form known-answer tests (test_oracle_kat.py).

Exact float32 semantics without a float32 FPU:
* +, -, *, /, sqrt of float32 operands evaluated in float64 and rounded once
  to float32 are correctly rounded (53 >= 2*24 + 2, Figueroa 1995), so plain
  Python floats + :func:`f32` reproduce IEEE binary32 exactly;
* fmaf needs one rounding of a*b + c: the product is exact in float64, the sum
  is made exact with TwoSum and the float32 rounding corrected at ties (:func:`fmaf`);
* numpy float32 array arithmetic is IEEE binary32 per element (no contraction).
"""
from __future__ import annotations

import math
import struct

import numpy as np

_pack, _unpack = struct.Struct("<f").pack, struct.Struct("<f").unpack


def f32(x: float) -> float:
    """Round a Python float to the nearest binary32 (ties to even)."""
    return _unpack(_pack(x))[0]


def _next32(x: float, up: bool) -> float:
    return float(np.nextafter(np.float32(x), np.float32(np.inf if up else -np.inf)))


def fmaf(a: float, b: float, c: float) -> float:
    """Correctly rounded binary32 fused multiply-add of binary32 values."""
    p = a * b                       # exact in binary64
    s = p + c
    bb = s - p
    err = (p - (s - bb)) + (c - bb)  # TwoSum: p + c == s + err exactly
    r = f32(s)
    if err == 0.0 or r == s:
        return r
    lo, hi = (r, _next32(r, True)) if r < s else (_next32(r, False), r)
    if s - lo == hi - s:            # s sits exactly on a binary32 midpoint
        return hi if err > 0 else lo
    return r


# ---------------------------------------------------------------------------
# constants (include/vct_spec.h)
# ---------------------------------------------------------------------------
ALPHA_STOP, STEP_SCALE, SQRT3 = f32(0.95), 0.5, f32(1.7320508)
TAU_MIN, TAU_MAX = f32(0.02), 1.0
TAN30, TAN20 = f32(0.577350259), f32(0.36397022)
LOG2_SQRT2, INV_LN2 = f32(1.41421354), f32(1.44269502)
C9, C7, C5, C3 = f32(0.111111112), f32(0.142857149), f32(0.200000003), f32(0.333333343)
S45, W0, WK = f32(0.707106769), f32(0.150221109), f32(0.106222361)
CONES9 = [(1.0, 0.0, 0.0, W0)] + [
    (S45, ct, cb, WK) for ct, cb in
    [(S45, 0.0), (0.5, 0.5), (0.0, S45), (-0.5, 0.5), (-S45, 0.0), (-0.5, -0.5), (0.0, -S45), (0.5, -0.5)]]
CONES1 = [(1.0, 0.0, 0.0, 1.0)]


def log2(x: float) -> float:
    bits = struct.unpack("<I", _pack(x))[0]
    e = ((bits >> 23) & 0xFF) - 127
    f = struct.unpack("<f", struct.pack("<I", (bits & 0x007FFFFF) | 0x3F800000))[0]
    if f > LOG2_SQRT2:
        f = f32(f * 0.5)
        e += 1
    s = f32(f32(f - 1.0) / f32(f + 1.0))
    z = f32(s * s)
    p = C9
    for c in (C7, C5, C3, 1.0):
        p = fmaf(p, z, c)
    ln = f32(f32(2.0 * s) * p)
    return fmaf(ln, INV_LN2, float(e))


# ---------------------------------------------------------------------------
# K1 voxelization (numpy float32, vectorised over candidate voxels)
# ---------------------------------------------------------------------------
F = np.float32


def _dot(ux, uy, uz, vx, vy, vz):
    return (ux * vx + uy * vy) + uz * vz


def _sat(q, cx, cy, cz):
    """q: (3,3) float32 voxel-unit vertices; c*: float32 arrays of voxel centres."""
    a = [(F(q[k, 0]) - cx, F(q[k, 1]) - cy, F(q[k, 2]) - cz) for k in range(3)]
    ok = np.ones(cx.shape, bool)
    h = F(0.5)
    for ax in range(3):
        mn = np.fmin(np.fmin(a[0][ax], a[1][ax]), a[2][ax])
        mx = np.fmax(np.fmax(a[0][ax], a[1][ax]), a[2][ax])
        ok &= ~((mn > h) | (mx < -h))
    e = [tuple(a[(i + 1) % 3][c] - a[i][c] for c in range(3)) for i in range(3)]
    nx = e[0][1] * e[1][2] - e[0][2] * e[1][1]
    ny = e[0][2] * e[1][0] - e[0][0] * e[1][2]
    nz = e[0][0] * e[1][1] - e[0][1] * e[1][0]
    vmin = [np.where(n > 0, -h - a[0][c], h - a[0][c]) for c, n in enumerate((nx, ny, nz))]
    vmax = [np.where(n > 0, h - a[0][c], -h - a[0][c]) for c, n in enumerate((nx, ny, nz))]
    ok &= ~(_dot(nx, ny, nz, *vmin) > 0)
    ok &= _dot(nx, ny, nz, *vmax) >= 0
    z0 = np.zeros_like(cx)
    for ex, ey, ez in e:
        for ux, uy, uz in ((z0, -ez, ey), (ez, z0, -ex), (-ey, ex, z0)):
            p = [_dot(ux, uy, uz, *a[k]) for k in range(3)]
            rad = h * ((np.abs(ux) + np.abs(uy)) + np.abs(uz))
            mn = np.fmin(np.fmin(p[0], p[1]), p[2])
            mx = np.fmax(np.fmax(p[0], p[1]), p[2])
            ok &= ~((mn > rad) | (mx < -rad))
    return ok


def _roundf(x):
    x = np.asarray(x, np.float64)
    return (np.sign(x) * np.floor(np.abs(x) + 0.5)).astype(np.int64)


# ---- diffuse maps (include/vct_spec.h "diffuse maps"), scalar binary32 -----------
def _lerp(a, b, f):
    return fmaf(f, f32(b - a), a)


def tex_sample(t, u, v):
    """T(u, v).rgb of an (H, W, 4) uint8 texture: GL_REPEAT, bilinear, texel centres."""
    H, W = t.shape[:2]
    u = float(u) if math.isfinite(u) else 0.0
    v = float(v) if math.isfinite(v) else 0.0
    fu, fv = f32(u - math.floor(u)), f32(v - math.floor(v))
    s, tt = f32(f32(fu * W) - 0.5), f32(f32(fv * H) - 0.5)
    sx, sy = math.floor(s), math.floor(tt)
    ax, ay = f32(s - sx), f32(tt - sy)
    x0, y0 = int(sx) % W, int(sy) % H
    x1, y1 = (int(sx) + 1) % W, (int(sy) + 1) % H
    px = lambda y, x, c: f32(float(t[y, x, c]) / 255.0)
    return [_lerp(_lerp(px(y0, x0, c), px(y0, x1, c), ax), _lerp(px(y1, x0, c), px(y1, x1, c), ax), ay)
            for c in range(3)]


def _dot32(a, b):
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def tri_bary(q0, q1, q2, c):
    e1 = [f32(q1[k] - q0[k]) for k in range(3)]
    e2 = [f32(q2[k] - q0[k]) for k in range(3)]
    w = [f32(c[k] - q0[k]) for k in range(3)]
    d11, d12, d22 = _dot32(e1, e1), _dot32(e1, e2), _dot32(e2, e2)
    w1, w2 = _dot32(w, e1), _dot32(w, e2)
    den = f32(f32(d11 * d22) - f32(d12 * d12))
    b1 = b2 = 0.0
    if den > 0:
        b1 = f32(f32(f32(d22 * w1) - f32(d12 * w2)) / den)
        b2 = f32(f32(f32(d11 * w2) - f32(d12 * w1)) / den)
    b1, b2 = max(b1, 0.0), max(b2, 0.0)
    s = f32(b1 + b2)
    if s > 1.0:
        b1, b2 = f32(b1 / s), f32(b2 / s)
    return b1, b2


def tri_uv(uv, b1, b2):
    return tuple(fmaf(b2, f32(uv[4 + k] - uv[k]), fmaf(b1, f32(uv[2 + k] - uv[k]), uv[k])) for k in range(2))


def voxelize(n, g0, extent, verts, idx, tri_mat=None, kd4=None, mat_map=None, textures=(), uv_offset=24):
    g0 = np.asarray(g0, F)
    inv_h = F(n) / F(extent)
    sums = np.zeros((n ** 3, 6), np.int64)
    counts = np.zeros(n ** 3, np.int64)
    idx = np.asarray(idx).reshape(-1, 3)
    for t, tri in enumerate(idx):
        p = np.asarray(verts, F)[tri, :3]
        q = (p - g0) * inv_h
        e1, e2 = p[1] - p[0], p[2] - p[0]
        fn = np.array([e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                       e1[0] * e2[1] - e1[1] * e2[0]], F)
        ln = np.sqrt(_dot(*fn, *fn))
        fn = fn / ln if ln > 0 else np.zeros(3, F)
        m = 0 if tri_mat is None else int(tri_mat[t])
        kd = np.ones(3, F) if kd4 is None else np.asarray(kd4, F)[m, :3]
        fix = np.concatenate([_roundf(kd * F(65536)), _roundf(fn * F(65536))])
        lo, hi = [], []
        for a in range(3):
            mn, mx = np.fmin(np.fmin(q[0, a], q[1, a]), q[2, a]), np.fmax(np.fmax(q[0, a], q[1, a]), q[2, a])
            lo.append(max(0, int(np.ceil(np.fmax(mn, F(-1)))) - 1))
            hi.append(min(n - 1, int(np.floor(np.fmin(mx, F(n) + F(1))))))
        if any(l > h for l, h in zip(lo, hi)):
            continue
        zz, yy, xx = np.meshgrid(*[np.arange(lo[a], hi[a] + 1) for a in (2, 1, 0)], indexing="ij")
        c = [ar.astype(F) + F(0.5) for ar in (xx, yy, zz)]
        hit = _sat(q, *c)
        v = (xx + n * (yy + n * zz))[hit]
        tex = -1 if mat_map is None else int(mat_map[m])
        if tex < 0:
            np.add.at(sums, v, fix[None, :])
        else:   # albedo = Kd x T(uv at the voxel centre's projection), per covered voxel
            uvf = np.asarray(verts, F)[tri, uv_offset // 4: uv_offset // 4 + 2].reshape(-1)
            uv = [float(x) for x in uvf]
            qf = [[float(x) for x in q[k]] for k in range(3)]
            for vx, vy, vz, vi in zip(xx[hit], yy[hit], zz[hit], v):
                b1, b2 = tri_bary(qf[0], qf[1], qf[2], (vx + 0.5, vy + 0.5, vz + 0.5))
                tu, tv = tri_uv(uv, b1, b2)
                rgb = tex_sample(textures[tex], tu, tv)
                f = [int(_roundf(f32(f32(float(kd[k]) * rgb[k]) * 65536.0))) for k in range(3)]
                sums[vi, :3] += f
                sums[vi, 3:] += fix[3:]
        np.add.at(counts, v, 1)
    return sums, counts.astype(np.uint32)


def resolve(n, sums, counts):
    ao = np.zeros((n ** 3, 4), F)
    nm = np.zeros((n ** 3, 4), F)
    occ = counts > 0
    den = counts[occ].astype(np.float64) * 65536.0
    ao[occ, :3] = (sums[occ, :3].astype(np.float64) / den[:, None]).astype(F)
    ao[occ, 3] = 1
    s = sums[occ, 3:].astype(np.float64)
    ln = np.sqrt((s[:, 0] * s[:, 0] + s[:, 1] * s[:, 1]) + s[:, 2] * s[:, 2])
    out = np.zeros_like(s)
    nz = ln > 0
    out[nz] = s[nz] / ln[nz, None]
    nm[occ, :3] = out.astype(F)
    return ao.reshape(n, n, n, 4), nm.reshape(n, n, n, 4)


# ---------------------------------------------------------------------------
# K2 injection (pure Python DDA)
# ---------------------------------------------------------------------------
def inject(n, ao, nm, light, color=(1.0, 1.0, 1.0)):
    lx, ly, lz = (f32(v) for v in light)
    ln = f32(math.sqrt(f32(f32(f32(lx * lx) + f32(ly * ly)) + f32(lz * lz))))
    lx, ly, lz = f32(lx / ln), f32(ly / ln), f32(lz / ln)
    occ = ao[..., 3] != 0
    r0 = np.zeros((n, n, n, 4), F)
    inf = math.inf
    for z, y, x in zip(*np.nonzero(occ)):
        nx, ny, nz_ = (float(v) for v in nm[z, y, x, :3])
        ndl = f32(f32(f32(nx * lx) + f32(ny * ly)) + f32(nz_ * lz))
        L = [0.0, 0.0, 0.0]
        if ndl > 0:
            q = [f32(f32(x + 0.5) + nx), f32(f32(y + 0.5) + ny), f32(f32(z + 0.5) + nz_)]
            l = (lx, ly, lz)
            v = [math.floor(c) for c in q]
            vis = 1.0
            if all(0 <= c < n for c in v):
                st = [1 if c > 0 else (-1 if c < 0 else 0) for c in l]
                td = [f32(1.0 / abs(l[i])) if st[i] else inf for i in range(3)]
                tm = [f32(f32(float(v[i] + 1) - q[i]) * td[i]) if st[i] > 0 else
                      (f32(f32(q[i] - float(v[i])) * td[i]) if st[i] < 0 else inf) for i in range(3)]
                while True:
                    if occ[v[2], v[1], v[0]]:
                        vis = 0.0
                        break
                    if tm[0] <= tm[1] and tm[0] <= tm[2]:
                        a = 0
                    elif tm[1] <= tm[2]:
                        a = 1
                    else:
                        a = 2
                    v[a] += st[a]
                    if not 0 <= v[a] < n:
                        break
                    tm[a] = f32(tm[a] + td[a])
            L = [f32(f32(f32(float(ao[z, y, x, c]) * f32(color[c])) * ndl) * vis) for c in range(3)]
        r0[z, y, x] = (L[0], L[1], L[2], 1.0)
    return r0


# ---------------------------------------------------------------------------
# K3 mips (numpy float32)
# ---------------------------------------------------------------------------
def _down(src, aniso_face):
    n2 = src.shape[0] // 2
    C = src.reshape(n2, 2, n2, 2, n2, 2, 4)      # [z, dz, y, dy, x, dx, c]
    acc = np.zeros((n2, n2, n2, 4), F)
    if aniso_face is None:
        for dz in range(2):
            for dy in range(2):
                for dx in range(2):
                    acc = acc + C[:, dz, :, dy, :, dx, :]
        return acc * F(0.125)
    axis, fr = aniso_face >> 1, aniso_face & 1
    bk = 1 - fr
    for r1 in range(2):
        for r0 in range(2):
            if axis == 0:
                f, b = C[:, r1, :, r0, :, fr, :], C[:, r1, :, r0, :, bk, :]
            elif axis == 1:
                f, b = C[:, r1, :, fr, :, r0, :], C[:, r1, :, bk, :, r0, :]
            else:
                f, b = C[:, fr, :, r1, :, r0, :], C[:, bk, :, r1, :, r0, :]
            oma = F(1) - f[..., 3:4]
            acc = acc + (f + oma * b)
    return acc * F(0.25)


def build_mips(r0, aniso=True):
    """-> {level: [face volumes]} for levels 1..L"""
    n = r0.shape[0]
    L = int(round(math.log2(n)))
    out = {}
    faces = 6 if aniso else 1
    for l in range(1, L + 1):
        out[l] = [_down(r0 if l == 1 else out[l - 1][f], f if aniso else None) for f in range(faces)]
    return out


# ---------------------------------------------------------------------------
# K4 cone trace (pure Python, exact binary32; a handful of pixels)
# ---------------------------------------------------------------------------
class Tracer:
    def __init__(self, n, g0, extent, r0, mips, aniso=True):
        self.n, self.L = n, int(round(math.log2(n)))
        self.g0 = [f32(v) for v in g0]
        self.inv_h = f32(f32(n) / f32(extent))
        self.r0, self.mips, self.aniso = r0, mips, aniso
        self.tmax = f32(f32(n) * SQRT3)

    def _tri(self, vol, q, scale):
        nl = vol.shape[0]
        c = [f32(f32(q[i] * scale) - 0.5) for i in range(3)]
        fl = [float(math.floor(v)) for v in c]
        i0 = [int(v) for v in fl]
        fr = [f32(c[i] - fl[i]) for i in range(3)]
        w = [(f32(1.0 - fr[i]), fr[i]) for i in range(3)]
        acc = [0.0, 0.0, 0.0, 0.0]
        for dz in range(2):
            for dy in range(2):
                for dx in range(2):
                    x, y, z = i0[0] + dx, i0[1] + dy, i0[2] + dz
                    if not (0 <= x < nl and 0 <= y < nl and 0 <= z < nl):
                        continue
                    wc = f32(f32(w[0][dx] * w[1][dy]) * w[2][dz])
                    t = vol[z, y, x]
                    acc = [fmaf(wc, float(t[k]), acc[k]) for k in range(4)]
        return acc

    def _tri_dir(self, vols, q, scale, wd):
        """directional sample: faces combined per corner texel, then trilinear"""
        nl = vols[0].shape[0]
        c = [f32(f32(q[i] * scale) - 0.5) for i in range(3)]
        fl = [float(math.floor(v)) for v in c]
        i0 = [int(v) for v in fl]
        fr = [f32(c[i] - fl[i]) for i in range(3)]
        w = [(f32(1.0 - fr[i]), fr[i]) for i in range(3)]
        acc = [0.0, 0.0, 0.0, 0.0]
        for dz in range(2):
            for dy in range(2):
                for dx in range(2):
                    x, y, z = i0[0] + dx, i0[1] + dy, i0[2] + dz
                    if not (0 <= x < nl and 0 <= y < nl and 0 <= z < nl):
                        continue
                    wc = f32(f32(w[0][dx] * w[1][dy]) * w[2][dz])
                    tx, ty, tz = (vols[f][z, y, x] for f in range(3))
                    for k in range(4):
                        v = f32(wd[0] * float(tx[k]))
                        v = fmaf(wd[1], float(ty[k]), v)
                        v = fmaf(wd[2], float(tz[k]), v)
                        acc[k] = fmaf(wc, v, acc[k])
        return acc

    def _level(self, l, q, faces, wd):
        scale = 2.0 ** -l
        if l == 0:
            return self._tri(self.r0, q, 1.0)
        if not self.aniso:
            return self._tri(self.mips[l][0], q, scale)
        return self._tri_dir([self.mips[l][faces[i]] for i in range(3)], q, scale, wd)

    def march(self, o, d, tau):
        tau2 = f32(2.0 * tau)
        nf = float(self.n)
        faces = [0 if d[0] >= 0 else 1, 2 if d[1] >= 0 else 3, 4 if d[2] >= 0 else 5]
        wd = [f32(v * v) for v in d]
        c, a, t, steps = [0.0, 0.0, 0.0], 0.0, 1.0, 0
        while True:
            if not a < ALPHA_STOP or not t <= self.tmax:
                break
            q = [f32(o[i] + f32(d[i] * t)) for i in range(3)]
            if not all(0.0 <= v <= nf for v in q):
                break
            D = max(1.0, f32(tau2 * t))
            m = min(log2(D), float(self.L))
            l0 = int(m)
            fr = f32(m - l0)
            s = self._level(l0, q, faces, wd)
            if fr > 0 and l0 < self.L:
                s1 = self._level(l0 + 1, q, faces, wd)
                omf = f32(1.0 - fr)
                s = [fmaf(fr, s1[k], f32(omf * s[k])) for k in range(4)]
            oma = f32(1.0 - a)
            c = [fmaf(oma, s[k], c[k]) for k in range(3)]
            a = fmaf(oma, s[3], a)
            t = f32(t + f32(STEP_SCALE * D))
            steps += 1
        return c + [a], steps

    def pixel(self, P, N, rough, eye, cones=CONES9, tau_d=TAN30, specular=True):
        if P[3] == 0:
            return [0.0] * 4, [0.0] * 4, 0
        nx, ny, nz = (float(v) for v in N[:3])
        o = [f32(f32(f32(float(P[i]) - self.g0[i]) * self.inv_h) + float(N[i])) for i in range(3)]
        sgn = math.copysign(1.0, nz)
        ka = f32(-1.0 / f32(sgn + nz))
        kb = f32(f32(nx * ny) * ka)
        T = [f32(1.0 + f32(f32(f32(sgn * nx) * nx) * ka)), f32(sgn * kb), -f32(sgn * nx)]
        B = [kb, f32(sgn + f32(f32(ny * ny) * ka)), -ny]
        irr, occ, steps = [0.0, 0.0, 0.0], 0.0, 0
        for cn, ct, cb, wk in cones:
            d = [f32(f32(f32(cn * n_) + f32(ct * t_)) + f32(cb * b_)) for n_, t_, b_ in
                 zip((nx, ny, nz), T, B)]
            res, st = self.march(o, d, tau_d)
            steps += st
            irr = [fmaf(wk, res[k], irr[k]) for k in range(3)]
            occ = fmaf(wk, res[3], occ)
        diff = irr + [f32(1.0 - occ)]
        spec = [0.0] * 4
        if specular:
            v = [f32(float(eye[i]) - float(P[i])) for i in range(3)]
            vl = f32(math.sqrt(f32(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2]))))
            v = [f32(x / vl) for x in v]
            ndv = f32(f32(f32(nx * v[0]) + f32(ny * v[1])) + f32(nz * v[2]))
            k2 = f32(2.0 * ndv)
            r = [f32(f32(k2 * n_) - v_) for n_, v_ in zip((nx, ny, nz), v)]
            tau = min(max(float(rough), TAU_MIN), TAU_MAX)
            spec, st = self.march(o, r, tau)
            steps += st
        return diff, spec, steps
