"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  The product path (voxel-based-global-illumination_amd/)
never does.  See vct_oracle.h for provenance: the reference holds no
implementation of this path, so the oracle restates SURVEY.md Appendix A and
is pinned by closed-form known-answer tests (tests/test_oracle_kat.py).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle_vct.so")
CPU_BACKEND = os.path.join(HERE, "_build", "libvct_cpu.so")   # include/vct.h on the oracle


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


class _Texture(C.Structure):
    _fields_ = [("rgba8", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32)]


def _tex_array(textures):
    """list of (H, W, 4) uint8 arrays -> (ctypes array of vo_texture, keep-alive list)"""
    keep = [np.ascontiguousarray(t, np.uint8) for t in textures]
    arr = (_Texture * max(len(keep), 1))()
    for i, t in enumerate(keep):
        assert t.ndim == 3 and t.shape[2] == 4, t.shape
        arr[i].rgba8 = t.ctypes.data_as(C.c_void_p)
        arr[i].height, arr[i].width = t.shape[0], t.shape[1]
    return arr, keep


class _TraceParams(C.Structure):
    _fields_ = [("n", C.c_uint32), ("g0", C.c_float * 3), ("extent", C.c_float), ("aniso", C.c_int),
                ("n_diffuse", C.c_uint32), ("specular", C.c_uint32), ("eye", C.c_float * 3)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.c_void_p
        L.vo_pyramid_floats.restype = C.c_size_t
        L.vo_pyramid_floats.argtypes = [C.c_uint32, C.c_int]
        L.vo_level_offset.restype = C.c_size_t
        L.vo_level_offset.argtypes = [C.c_uint32, C.c_int, C.c_uint32]
        L.vo_voxelize.restype = C.c_int
        L.vo_voxelize.argtypes = [C.c_uint32, P, C.c_float, P, C.c_uint32, C.c_uint32, P, C.c_uint32,
                                  P, P, C.c_uint32, P, P]
        L.vo_voxelize_tex.restype = C.c_int
        L.vo_voxelize_tex.argtypes = [C.c_uint32, P, C.c_float, P, C.c_uint32, C.c_uint32, P, C.c_uint32,
                                      P, P, C.c_uint32, P, C.c_uint32, P, C.c_uint32, P, P]
        L.vo_tex_sample.restype = None
        L.vo_tex_sample.argtypes = [C.POINTER(_Texture), C.c_float, C.c_float, P]
        L.vo_tri_bary.restype = None
        L.vo_tri_bary.argtypes = [P, P, P, P, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.vo_tri_uv.restype = None
        L.vo_tri_uv.argtypes = [P, C.c_float, C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.vo_resolve.restype = None
        L.vo_resolve.argtypes = [C.c_uint32, P, P, P, P]
        L.vo_inject.restype = None
        L.vo_inject.argtypes = [C.c_uint32, P, P, P, P, P]
        L.vo_build_mips.restype = None
        L.vo_build_mips.argtypes = [C.c_uint32, C.c_int, P, P]
        L.vo_trace.restype = C.c_uint64
        L.vo_trace.argtypes = [C.POINTER(_TraceParams), P, P, P, P, P, C.c_uint32, C.c_uint32, C.c_uint32,
                               P, P, P, C.c_int]
        L.vo_composite.restype = None
        L.vo_composite.argtypes = [C.c_uint32, P, C.c_float, P, P, P, P, P, P, C.c_uint32, C.c_uint32, P, P, P, P]
        L.vo_log2.restype = C.c_float
        L.vo_log2.argtypes = [C.c_float]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def log2(x: float) -> float:
    return float(lib().vo_log2(C.c_float(x)))


def voxelize(n, aabb_min, extent, verts, idx, tri_mat=None, kd4=None, mat_map=None, textures=(), uv_offset=24):
    """-> (sums6 [n^3,6] int64, counts [n^3] uint32).  mat_map (per material: texture
    index or -1) + textures ((H, W, 4) uint8) select the diffuse-map rule (vo_voxelize_tex)."""
    verts = np.ascontiguousarray(verts, np.float32)
    idx = np.ascontiguousarray(idx, np.uint32).reshape(-1)
    mat = None if tri_mat is None else np.ascontiguousarray(tri_mat, np.uint32)
    kd = None if kd4 is None else np.ascontiguousarray(kd4, np.float32).reshape(-1, 4)
    mm = None if mat_map is None else np.ascontiguousarray(mat_map, np.int32).reshape(-1)
    n_mat = kd.shape[0] if kd is not None else (mm.size if mm is not None else 0)
    g0 = np.asarray(aabb_min, np.float32)
    sums = np.zeros((n ** 3, 6), np.int64)
    counts = np.zeros(n ** 3, np.uint32)
    tarr, keep = _tex_array(textures)
    rc = lib().vo_voxelize_tex(n, _p(g0), C.c_float(extent), _p(verts), verts.shape[1] * 4, verts.shape[0],
                               _p(idx), idx.size, _p(mat), _p(kd), n_mat, _p(mm), uv_offset,
                               C.cast(tarr, C.c_void_p), len(keep), _p(sums), _p(counts))
    if rc != 0:
        raise ValueError("oracle voxelize: index out of range")
    return sums, counts


def tex_sample(texture, u, v):
    """vct_spec.h T(u, v).rgb of one (H, W, 4) uint8 texture -> float32[3]"""
    tarr, keep = _tex_array([texture])
    out = np.zeros(3, np.float32)
    lib().vo_tex_sample(tarr, C.c_float(u), C.c_float(v), _p(out))
    return out


def tri_bary(q0, q1, q2, c):
    b1, b2 = C.c_float(), C.c_float()
    f = lambda a: np.ascontiguousarray(a, np.float32)
    q0, q1, q2, c = f(q0), f(q1), f(q2), f(c)
    lib().vo_tri_bary(_p(q0), _p(q1), _p(q2), _p(c), C.byref(b1), C.byref(b2))
    return b1.value, b2.value


def tri_uv(uv6, b1, b2):
    u, v = C.c_float(), C.c_float()
    lib().vo_tri_uv(_p(np.ascontiguousarray(uv6, np.float32)), C.c_float(b1), C.c_float(b2), C.byref(u), C.byref(v))
    return u.value, v.value


def resolve(n, sums, counts):
    ao = np.empty((n, n, n, 4), np.float32)
    nm = np.empty((n, n, n, 4), np.float32)
    lib().vo_resolve(n, _p(np.ascontiguousarray(sums)), _p(np.ascontiguousarray(counts)), _p(ao), _p(nm))
    return ao, nm


def inject(n, albedo_occ, normal, dir_to_light, color=(1.0, 1.0, 1.0)):
    r0 = np.empty((n, n, n, 4), np.float32)
    l = np.asarray(dir_to_light, np.float32)
    c = np.asarray(color, np.float32)
    lib().vo_inject(n, _p(np.ascontiguousarray(albedo_occ, np.float32)),
                    _p(np.ascontiguousarray(normal, np.float32)), _p(l), _p(c), _p(r0))
    return r0


def build_mips(n, r0, aniso=True):
    """-> flat pyramid (levels 1..L) float32"""
    pyr = np.empty(lib().vo_pyramid_floats(n, 1 if aniso else 0), np.float32)
    lib().vo_build_mips(n, 1 if aniso else 0, _p(np.ascontiguousarray(r0, np.float32)), _p(pyr))
    return pyr


def pyramid_levels(n, pyr, aniso=True):
    """flat pyramid -> [level][face] (n_l, n_l, n_l, 4) views (level index starts at 1)"""
    L = int(np.log2(n))
    faces = 6 if aniso else 1
    out = {}
    for l in range(1, L + 1):
        nl = n >> l
        off = lib().vo_level_offset(n, 1 if aniso else 0, l)
        vol = pyr[off: off + faces * nl ** 3 * 4].reshape(faces, nl, nl, nl, 4)
        out[l] = [vol[f] for f in range(faces)]
    return out


def trace(n, aabb_min, extent, r0, pyr, pos4, nrm4, alb4, eye, aniso=True, n_diffuse=9, specular=True,
          row_step=1, threads=0):
    """-> dict(diffuse, spec, steps_px, cone_steps); rows y % row_step != 0 are left zero."""
    h, w = pos4.shape[:2]
    p = _TraceParams()
    p.n = n
    p.g0 = (C.c_float * 3)(*[float(x) for x in aabb_min])
    p.extent = float(extent)
    p.aniso = 1 if aniso else 0
    p.n_diffuse = n_diffuse
    p.specular = 1 if specular else 0
    p.eye = (C.c_float * 3)(*[float(x) for x in eye])
    diff = np.zeros((h, w, 4), np.float32)
    spec = np.zeros((h, w, 4), np.float32)
    steps = np.zeros((h, w), np.uint32)
    tot = lib().vo_trace(C.byref(p), _p(np.ascontiguousarray(r0, np.float32)), _p(pyr),
                         _p(np.ascontiguousarray(pos4, np.float32)), _p(np.ascontiguousarray(nrm4, np.float32)),
                         _p(np.ascontiguousarray(alb4, np.float32)), w, h, row_step,
                         _p(diff), _p(spec), _p(steps), threads)
    return {"diffuse": diff, "spec": spec, "steps_px": steps, "cone_steps": int(tot)}


def composite(n, aabb_min, extent, albedo_occ, pos4, nrm4, alb4, diffuse4, spec4, dir_to_light,
              color=(1.0, 1.0, 1.0)):
    """f3 composite (vct_spec.h) -> (linear float4 [h][w][4], rgba8 uint32 [h][w])."""
    h, w = pos4.shape[:2]
    lin = np.empty((h, w, 4), np.float32)
    rgba = np.empty((h, w), np.uint32)
    f32 = lambda a: np.ascontiguousarray(a, np.float32)
    lib().vo_composite(n, _p(f32(aabb_min)), float(extent), _p(f32(albedo_occ)), _p(f32(pos4)), _p(f32(nrm4)),
                       _p(f32(alb4)), _p(f32(diffuse4)), _p(f32(spec4)), w, h, _p(f32(dir_to_light)),
                       _p(f32(color)), _p(lin), _p(rgba))
    return lin, rgba


def pipeline(n, aabb_min, extent, verts, idx, tri_mat, kd4, light_dir, light_color=(1, 1, 1), aniso=True,
             mat_map=None, textures=()):
    """K1 -> resolve -> K2 -> K3 on the CPU.  -> dict of every intermediate."""
    sums, counts = voxelize(n, aabb_min, extent, verts, idx, tri_mat, kd4, mat_map, textures)
    ao, nm = resolve(n, sums, counts)
    r0 = inject(n, ao, nm, light_dir, light_color)
    pyr = build_mips(n, r0, aniso)
    return {"sums": sums, "counts": counts, "albedo_occ": ao, "normal": nm, "r0": r0, "pyr": pyr}
