"""ctypes binding of include/vct_host.h (libvct_host.so: the C++ host's scene loader,
camera and placement helpers; CPU only).  Test infrastructure."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "voxel-based-global-illumination_amd")
LIB = os.path.join(PKG, "vct", "libvct_host.so")
_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", PKG, "vct/libvct_host.so"], check=True, capture_output=True)
    lib = C.CDLL(LIB)
    P, F = C.c_void_p, C.POINTER(C.c_float)
    lib.vcth_load_obj.argtypes = [C.c_char_p, C.POINTER(P), C.c_char_p, C.c_int]
    lib.vcth_num_meshes.argtypes = [P]
    lib.vcth_num_meshes.restype = C.c_uint32
    lib.vcth_num_materials.argtypes = [P]
    lib.vcth_num_materials.restype = C.c_uint32
    lib.vcth_mesh.argtypes = [P, C.c_uint32, C.POINTER(P), C.POINTER(C.c_uint32), C.POINTER(P),
                              C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    lib.vcth_material.argtypes = [P, C.c_uint32, C.POINTER(C.c_char_p), F, F, F]
    lib.vcth_free.argtypes = [P]
    lib.vcth_transform.argtypes = [P, F]
    lib.vcth_transform.restype = None
    lib.vcth_bounds.argtypes = [P, F, F]
    lib.vcth_reference_model_matrix.argtypes = [F]
    lib.vcth_reference_model_matrix.restype = None
    lib.vcth_grid_for_bounds.argtypes = [F, F, C.c_uint32, F, F]
    lib.vcth_grid_for_bounds.restype = None
    lib.vcth_camera_eval.argtypes = [F, C.c_char_p, F, F, C.c_int, F]
    _lib = lib
    return lib


def fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def reference_model_matrix() -> np.ndarray:
    m = np.zeros(16, np.float32)
    load().vcth_reference_model_matrix(fptr(m))
    return m


def camera_eval(init, ops) -> np.ndarray:
    """Host Camera after `ops` [(kind, a, b)] -> float32[15] (Position, Front, Right, Up, Yaw, Pitch, Zoom)."""
    kinds = "".join(o[0] for o in ops).encode() or b"\0"
    a = np.array([o[1] for o in ops] or [0], np.float32)
    b = np.array([o[2] for o in ops] or [0], np.float32)
    out = np.zeros(15, np.float32)
    init = np.asarray(init, np.float32)
    assert load().vcth_camera_eval(fptr(init), kinds, fptr(a), fptr(b), len(ops), fptr(out)) == 0
    return out


def grid_for_bounds(lo, hi, n):
    lo, hi = np.asarray(lo, np.float32), np.asarray(hi, np.float32)
    g0, e = np.zeros(3, np.float32), np.zeros(1, np.float32)
    load().vcth_grid_for_bounds(fptr(lo), fptr(hi), n, fptr(g0), fptr(e))
    return g0, float(e[0])


def load_placed(path, model_matrix=None):
    """OBJ through the host loader, optionally moved by a model matrix -> (verts [V,14], idx, tri_mat, kd4, lo, hi)."""
    lib = load()
    h = C.c_void_p()
    err = C.create_string_buffer(256)
    if lib.vcth_load_obj(path.encode(), C.byref(h), err, 256) != 0:
        raise RuntimeError(err.value.decode())
    try:
        if model_matrix is not None:
            lib.vcth_transform(h, fptr(np.ascontiguousarray(model_matrix, np.float32)))
        lo, hi = np.zeros(3, np.float32), np.zeros(3, np.float32)
        assert lib.vcth_bounds(h, fptr(lo), fptr(hi)) == 0
        vs, ids, tms = [], [], []
        base = 0
        for i in range(lib.vcth_num_meshes(h)):
            vp, ip = C.c_void_p(), C.c_void_p()
            nv, ni, mat = C.c_uint32(), C.c_uint32(), C.c_uint32()
            assert lib.vcth_mesh(h, i, C.byref(vp), C.byref(nv), C.byref(ip), C.byref(ni), C.byref(mat)) == 0
            if nv.value:
                vs.append(np.ctypeslib.as_array(C.cast(vp, C.POINTER(C.c_float)), (nv.value * 14,)).reshape(-1, 14).copy())
            if ni.value:
                idx = np.ctypeslib.as_array(C.cast(ip, C.POINTER(C.c_uint32)), (ni.value,)).copy()
                ids.append(idx + base)
                tms.append(np.full(ni.value // 3, mat.value, np.uint32))
            base += nv.value
        kd = []
        for i in range(lib.vcth_num_materials(h)):
            name = C.c_char_p()
            ka, kdv, ks = (np.zeros(4, np.float32) for _ in range(3))
            lib.vcth_material(h, i, C.byref(name), fptr(ka), fptr(kdv), fptr(ks))
            kd.append(kdv)
        return (np.concatenate(vs), np.concatenate(ids), np.concatenate(tms), np.array(kd, np.float32), lo, hi)
    finally:
        lib.vcth_free(h)
