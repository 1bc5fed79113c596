"""vct — Python host mirror of the MI355X voxel-cone-tracing path.

The product is the C-ABI library ``libvct_hip.so`` (include/vct.h).  This
package is host plumbing around it, shaped like the reference's plug-in
surface:

* :class:`Context` wraps one ``vct_ctx`` (the state a reference ``Renderer``
  would own; renderer.h:3-10);
* :mod:`vct.camera` reproduces the reference FPS camera conventions
  (scene/camera.cpp:24-27, 73-83);
* :mod:`vct.scenes` builds synthetic scenes in the reference ``Vertex`` layout
  (include/stdafx.h:36-42, 56-byte records) with per-material Kd
  (scene/material.h:10), and the G-buffers of SURVEY.md 8d;
* :mod:`vct.renderer` is the ``Renderer`` / ``ConeTraceRenderer`` pair and the
  name-keyed registry (core/assets.h:17-20, assets.cpp:44, engine.cpp:151).

Host arrays are numpy; device arrays are torch tensors (torch is used only for
device memory, streams and torch.distributed).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import VctCamera, VctConfig, VctTraceArgs

__all__ = ["Context", "VctError", "VctConfig", "VctCamera", "tiles_for_rank", "VERTEX_FLOATS"]

VERTEX_FLOATS = 14          # reference Vertex: Position, Normal, TexCoords, Tangent, Bitangent
VERTEX_STRIDE = VERTEX_FLOATS * 4


class VctError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{_lib.STATUS.get(status, status)}: {msg}")
        self.status = status


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _f3(v):
    return (C.c_float * 3)(*[float(x) for x in v])


def tiles_for_rank(w: int, h: int, rank: int, world: int) -> int:
    return int(_lib.load().vct_tiles_for_rank(w, h, rank, world))


class Context:
    """One vct_ctx: grid + pyramid resident in HBM of one GPU."""

    def __init__(self, n: int, aabb_min, extent: float, aniso: bool = True, n_diffuse: int = 9,
                 specular: bool = True, device: int = -1, lib=None, devices: int = 0):
        # lib: another implementation of include/vct.h bound with _lib.bind (tests use
        # the CPU oracle backend); default: the in-tree HIP library, no fallback.
        # devices > 0: one context over that many GPUs (vct_create_multi; screen tiles
        # traced on every device, gathered on device 0 by peer copies)
        self.lib = lib if lib is not None else _lib.load()
        cfg = VctConfig()
        cfg.n = n
        cfg.aabb_min = (C.c_float * 3)(*[float(x) for x in aabb_min])
        cfg.extent = float(extent)
        cfg.aniso = 1 if aniso else 0
        cfg.n_diffuse = n_diffuse
        cfg.specular = 1 if specular else 0
        cfg.device = device
        h = C.c_void_p()
        if devices > 0:
            st = self.lib.vct_create_multi(C.byref(cfg), devices, C.byref(h))
        else:
            st = self.lib.vct_create(C.byref(cfg), C.byref(h))
        if st != 0:
            raise VctError(st, "vct_create failed (is a HIP device visible?)")
        self.num_devices = int(self.lib.vct_num_devices(h))
        self.h = h
        self.n = n
        self.aniso = aniso
        self.n_diffuse = n_diffuse
        self.specular = specular
        self.aabb_min = tuple(float(x) for x in aabb_min)
        self.extent = float(extent)

    # -- lifetime ---------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.vct_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st: int, what: str):
        if st != 0:
            err = self.lib.vct_last_error(self.h)
            raise VctError(st, f"{what}: {err.decode() if err else ''}")

    def set_stream(self, stream_ptr: int | None):
        self._check(self.lib.vct_set_stream(self.h, C.c_void_p(stream_ptr or 0)), "set_stream")

    def synchronize(self):
        self._check(self.lib.vct_synchronize(self.h), "synchronize")

    @property
    def num_levels(self) -> int:
        return int(self.lib.vct_num_levels(self.h))

    def level_dims(self, level: int):
        nl, nf = C.c_uint32(), C.c_uint32()
        self._check(self.lib.vct_level_dims(self.h, level, C.byref(nl), C.byref(nf)), "level_dims")
        return nl.value, nf.value

    # -- K1 / K2 / K3 -----------------------------------------------------
    def voxelize(self, verts: np.ndarray, idx: np.ndarray, tri_material: np.ndarray | None = None,
                 kd4: np.ndarray | None = None):
        verts = np.ascontiguousarray(verts, dtype=np.float32)
        assert verts.ndim == 2 and verts.shape[1] >= 3
        stride = verts.shape[1] * 4
        idx = np.ascontiguousarray(idx, dtype=np.uint32).reshape(-1)
        mat = None if tri_material is None else np.ascontiguousarray(tri_material, dtype=np.uint32)
        kd = None if kd4 is None else np.ascontiguousarray(kd4, dtype=np.float32).reshape(-1, 4)
        st = self.lib.vct_voxelize(self.h, _fptr(verts), stride, verts.shape[0], _fptr(idx), idx.size,
                                   _fptr(mat) if mat is not None else None,
                                   _fptr(kd) if kd is not None else None,
                                   0 if kd is None else kd.shape[0])
        self._check(st, "voxelize")

    def voxelize_device(self, verts, idx, tri_material=None, kd4=None):
        """K1 on device-resident torch tensors: verts [V, F] float32 (F >= 3, the
        56-byte Vertex is F = 14), idx [3T] int32/uint32, tri_material [T] int32,
        kd4 [M, 4] float32."""
        assert verts.dim() == 2 and verts.shape[1] >= 3 and verts.is_contiguous()
        ptr = lambda t: None if t is None else t.data_ptr()
        nm = 0 if kd4 is None else kd4.shape[0]
        st = self.lib.vct_voxelize_device(self.h, ptr(verts), verts.shape[1] * 4, verts.shape[0], ptr(idx),
                                          idx.numel(), ptr(tri_material), ptr(kd4), nm)
        self._check(st, "voxelize_device")

    def inject_directional(self, dir_to_light, color=(1.0, 1.0, 1.0)):
        l = (C.c_float * 3)(*[float(x) for x in dir_to_light])
        c = (C.c_float * 3)(*[float(x) for x in color])
        self._check(self.lib.vct_inject_directional(self.h, l, c), "inject")

    def build_mips(self):
        self._check(self.lib.vct_build_mips(self.h), "build_mips")

    # -- K4 ---------------------------------------------------------------
    def trace(self, pos4: np.ndarray, nrm4: np.ndarray, alb4: np.ndarray, eye, want_steps=True):
        h, w = pos4.shape[:2]
        pos4 = np.ascontiguousarray(pos4, dtype=np.float32)
        nrm4 = np.ascontiguousarray(nrm4, dtype=np.float32)
        alb4 = np.ascontiguousarray(alb4, dtype=np.float32)
        diff = np.empty((h, w, 4), np.float32)
        spec = np.empty((h, w, 4), np.float32)
        steps = np.empty((h, w), np.uint32) if want_steps else None
        total = C.c_uint64()
        st = self.lib.vct_trace(self.h, _fptr(pos4), _fptr(nrm4), _fptr(alb4), w, h, _f3(eye),
                                _fptr(diff), _fptr(spec), _fptr(steps) if steps is not None else None,
                                C.byref(total))
        self._check(st, "trace")
        return {"diffuse": diff, "spec": spec, "steps_px": steps, "cone_steps": int(total.value)}

    def trace_device(self, pos4, nrm4, alb4, width, height, eye, diffuse4, spec4, steps_px=None,
                     cone_steps=None, texel_fetches=None, tile_rank=0, tile_world=1, tile_compact=False,
                     variant=0):
        """Device-resident trace; arguments are torch CUDA tensors (or raw int pointers)."""
        a = VctTraceArgs()
        ptr = lambda t: None if t is None else (t if isinstance(t, int) else t.data_ptr())
        a.pos4, a.nrm4, a.alb4 = ptr(pos4), ptr(nrm4), ptr(alb4)
        a.width, a.height = width, height
        a.eye = _f3(eye)
        a.diffuse4, a.spec4 = ptr(diffuse4), ptr(spec4)
        a.steps_px, a.cone_steps = ptr(steps_px), ptr(cone_steps)
        a.texel_fetches = ptr(texel_fetches)
        a.tile_rank, a.tile_world = tile_rank, tile_world
        a.tile_compact = 1 if tile_compact else 0
        a.variant = variant
        self._check(self.lib.vct_trace_device(self.h, C.byref(a)), "trace_device")

    def untile_device(self, gathered4, width, height, world, frame4):
        ptr = lambda t: t if isinstance(t, int) else t.data_ptr()
        self._check(self.lib.vct_untile_device(self.h, ptr(gathered4), width, height, world, ptr(frame4)),
                    "untile_device")

    def untile_planes_device(self, gathered4, width, height, world, frames4):
        """gathered4: [world][planes][max_tiles*64*64][4]; frames4: sequence of [h][w][4] outputs."""
        ptr = lambda t: t if isinstance(t, int) else t.data_ptr()
        arr = (C.c_void_p * len(frames4))(*[ptr(f) for f in frames4])
        self._check(self.lib.vct_untile_planes_device(self.h, ptr(gathered4), len(frames4), width, height, world,
                                                      C.cast(arr, C.c_void_p)), "untile_planes_device")

    def gbuffer_raycast_device(self, cam, width, height, roughness, pos4, nrm4, alb4):
        c = cam.to_ctypes() if hasattr(cam, "to_ctypes") else cam
        ptr = lambda t: t if isinstance(t, int) else t.data_ptr()
        self._check(self.lib.vct_gbuffer_raycast_device(self.h, C.byref(c), width, height, float(roughness),
                                                        ptr(pos4), ptr(nrm4), ptr(alb4)), "raycast")

    def gbuffer_raster_device(self, cam, width, height, roughness, pos4, nrm4, alb4):
        """Row f2: tile-binned G-buffer pass (same output as gbuffer_raycast_device)."""
        c = cam.to_ctypes() if hasattr(cam, "to_ctypes") else cam
        ptr = lambda t: t if isinstance(t, int) else t.data_ptr()
        self._check(self.lib.vct_gbuffer_raster_device(self.h, C.byref(c), width, height, float(roughness),
                                                       ptr(pos4), ptr(nrm4), ptr(alb4)), "raster")

    def composite_device(self, pos4, nrm4, alb4, diffuse4, spec4, width, height, dir_to_light,
                         color=(1.0, 1.0, 1.0), out_linear4=None, out_rgba8=None):
        """Row f3 composite + present on device buffers (torch tensors or raw pointers)."""
        ptr = lambda t: None if t is None else (t if isinstance(t, int) else t.data_ptr())
        l = (C.c_float * 3)(*[float(x) for x in dir_to_light])
        c = (C.c_float * 3)(*[float(x) for x in color])
        self._check(self.lib.vct_composite_device(self.h, ptr(pos4), ptr(nrm4), ptr(alb4), ptr(diffuse4),
                                                  ptr(spec4), width, height, l, c, ptr(out_linear4),
                                                  ptr(out_rgba8)), "composite")

    # -- grid access ------------------------------------------------------
    def download_level(self, level: int, face: int = 0) -> np.ndarray:
        nl, _ = self.level_dims(level)
        out = np.empty((nl, nl, nl, 4), np.float32)
        self._check(self.lib.vct_download_level(self.h, level, face, _fptr(out)), "download_level")
        return out

    def download_pyramid(self) -> list:
        """[level][face] -> (n_l, n_l, n_l, 4) arrays (level 0 has one face)."""
        out = []
        for l in range(self.num_levels):
            _, nf = self.level_dims(l)
            out.append([self.download_level(l, f) for f in range(nf)])
        return out

    def upload_level0(self, r0: np.ndarray):
        r0 = np.ascontiguousarray(r0, dtype=np.float32)
        assert r0.size == self.n ** 3 * 4
        self._check(self.lib.vct_upload_level0(self.h, _fptr(r0)), "upload_level0")

    def level0_device(self):
        p, b = C.c_void_p(), C.c_size_t()
        self._check(self.lib.vct_level0_device(self.h, C.byref(p), C.byref(b)), "level0_device")
        return p.value, b.value

    def copy_level0_to_device(self, dst):
        ptr = dst if isinstance(dst, int) else dst.data_ptr()
        self._check(self.lib.vct_copy_level0_to_device(self.h, ptr), "copy_level0_to_device")

    def set_level0_from_device(self, src):
        ptr = src if isinstance(src, int) else src.data_ptr()
        self._check(self.lib.vct_set_level0_from_device(self.h, ptr), "set_level0_from_device")

    def download_voxels(self):
        n = self.n
        ao = np.empty((n, n, n, 4), np.float32)
        nm = np.empty((n, n, n, 4), np.float32)
        self._check(self.lib.vct_download_voxels(self.h, _fptr(ao), _fptr(nm)), "download_voxels")
        return ao, nm

    def download_accum(self):
        n = self.n
        sums = np.empty((n ** 3, 6), np.int64)
        counts = np.empty((n ** 3,), np.uint32)
        self._check(self.lib.vct_download_accum(self.h, _fptr(sums), _fptr(counts)), "download_accum")
        return sums, counts
