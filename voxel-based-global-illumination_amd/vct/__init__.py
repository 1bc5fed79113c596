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
* :mod:`vct.multi` splits the cone trace over ranks (screen tiles, RCCL
  broadcast of level 0, gather of the frame).
The ``Renderer`` / ``ConeTraceRenderer`` slot and the name-keyed registry
(core/assets.h:17-20, assets.cpp:44, engine.cpp:151) are in the C++ host
(``host/renderer.h``, ``host/assets.h``).

Host arrays are numpy; device arrays are torch tensors (torch is used only for
device memory, streams and torch.distributed).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib
from ._lib import VCT_ALL_RANKS, VctCamera, VctCommId, VctConfig, VctTexture, VctTraceArgs

__all__ = ["Context", "VctError", "VctConfig", "VctCamera", "tiles_for_rank", "tile_offset", "VERTEX_FLOATS",
           "VCT_ALL_RANKS", "comm_frame_layout"]

VERTEX_FLOATS = 14          # reference Vertex: Position, Normal, TexCoords, Tangent, Bitangent
VERTEX_STRIDE = VERTEX_FLOATS * 4
UV_OFFSET = 24              # offsetof(Vertex, TexCoords) (stdafx.h:36-42, mesh.cpp:49)


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


def tile_offset(w: int, h: int, rank: int, world: int) -> int:
    return int(_lib.load().vct_tile_offset(w, h, rank, world))


_EINVAL = 1
_F32 = ("torch.float32",)
_I32 = ("torch.int32", "torch.uint32")
_I64 = ("torch.int64", "torch.uint64")


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
        self.device = int(device)
        self.h = h
        self.n = n
        self.aniso = aniso
        self.n_diffuse = n_diffuse
        self.specular = specular
        self.aabb_min = tuple(float(x) for x in aabb_min)
        self.extent = float(extent)
        self.stream = 0          # the HIP stream of set_stream (0: the null stream)

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

    def _dev(self, t, name: str, dtypes=_F32, min_numel: int = 0):
        """Device pointer of a torch tensor after checking that the C-ABI may use it:
        a CUDA tensor on this context's device, of an accepted dtype, contiguous,
        with at least `min_numel` elements (an undersized output would be written
        out of bounds, a host tensor would fault the GPU).  None stays None; a raw
        int is taken as a device pointer the caller vouches for."""
        if t is None or isinstance(t, int):
            return t
        if not getattr(t, "is_cuda", False):
            raise VctError(_EINVAL, f"{name}: expected a device (cuda) tensor, got {getattr(t, 'device', type(t))}")
        if self.device >= 0 and t.device.index != self.device:
            raise VctError(_EINVAL, f"{name}: tensor on {t.device}, context on device {self.device}")
        if str(t.dtype) not in dtypes:
            raise VctError(_EINVAL, f"{name}: dtype {t.dtype}, expected one of {', '.join(dtypes)}")
        if not t.is_contiguous():
            raise VctError(_EINVAL, f"{name}: tensor is not contiguous")
        if t.numel() < min_numel:
            raise VctError(_EINVAL, f"{name}: {t.numel()} elements, needs at least {min_numel}")
        return t.data_ptr()

    def set_stream(self, stream_ptr: int | None):
        self._check(self.lib.vct_set_stream(self.h, C.c_void_p(stream_ptr or 0)), "set_stream")
        self.stream = stream_ptr or 0

    def synchronize(self):
        self._check(self.lib.vct_synchronize(self.h), "synchronize")

    @property
    def trace_form(self) -> int:
        """Kept candidate of the default cone trace for the current workload (vct_trace_form):
        bit 0 the form (0 union: bricks of up to six faces, 4 waves/SIMD; 1 occupancy, 5 waves/SIMD), bit 1
        ray reordering; -1 while still timing."""
        return int(self.lib.vct_trace_form(self.h))

    @property
    def num_levels(self) -> int:
        return int(self.lib.vct_num_levels(self.h))

    def level_dims(self, level: int):
        nl, nf = C.c_uint32(), C.c_uint32()
        self._check(self.lib.vct_level_dims(self.h, level, C.byref(nl), C.byref(nf)), "level_dims")
        return nl.value, nf.value

    # -- K1 / K2 / K3 -----------------------------------------------------
    def set_textures(self, textures):
        """Diffuse maps (vct_set_textures): a list of (H, W, 4) uint8 RGBA arrays, row 0 =
        the image's top row (stbi_load order); [] clears the set."""
        keep = [np.ascontiguousarray(t, dtype=np.uint8) for t in textures]
        arr = (VctTexture * max(len(keep), 1))()
        for i, t in enumerate(keep):
            if t.ndim != 3 or t.shape[2] != 4:
                raise VctError(_EINVAL, f"set_textures: texture {i} must be [H, W, 4] uint8, got {t.shape}")
            arr[i].rgba8 = t.ctypes.data_as(C.c_void_p)
            arr[i].height, arr[i].width = t.shape[0], t.shape[1]
        self._check(self.lib.vct_set_textures(self.h, C.cast(arr, C.c_void_p), len(keep)), "set_textures")

    def voxelize(self, verts: np.ndarray, idx: np.ndarray, tri_material: np.ndarray | None = None,
                 kd4: np.ndarray | None = None, material_map: np.ndarray | None = None,
                 uv_offset: int = UV_OFFSET):
        """K1 (vct_voxelize).  With material_map (per material: set_textures index or -1)
        it is vct_voxelize_textured: albedo = Kd x diffuse map at the hit's TexCoords."""
        verts = np.ascontiguousarray(verts, dtype=np.float32)
        assert verts.ndim == 2 and verts.shape[1] >= 3
        stride = verts.shape[1] * 4
        idx = np.ascontiguousarray(idx, dtype=np.uint32).reshape(-1)
        mat = None if tri_material is None else np.ascontiguousarray(tri_material, dtype=np.uint32).reshape(-1)
        kd = None if kd4 is None else np.ascontiguousarray(kd4, dtype=np.float32)
        mm = None if material_map is None else np.ascontiguousarray(material_map, dtype=np.int32).reshape(-1)
        if idx.size % 3:
            raise VctError(_EINVAL, f"voxelize: {idx.size} indices, not a multiple of 3")
        if mat is not None and mat.size != idx.size // 3:
            # vct_voxelize reads n_idx / 3 entries of tri_material
            raise VctError(_EINVAL, f"voxelize: tri_material has {mat.size} entries for {idx.size // 3} triangles")
        if kd is not None:
            if kd.ndim != 2 or kd.shape[1] != 4:
                raise VctError(_EINVAL, f"voxelize: kd4 must be [materials, 4], got {kd.shape}")
        n_mat = 0 if kd is None else kd.shape[0]
        if mm is None:
            st = self.lib.vct_voxelize(self.h, _fptr(verts), stride, verts.shape[0], _fptr(idx), idx.size,
                                       _fptr(mat) if mat is not None else None,
                                       _fptr(kd) if kd is not None else None, n_mat)
        else:
            if kd is not None and mm.size != n_mat:
                raise VctError(_EINVAL, f"voxelize: material_map has {mm.size} entries for {n_mat} materials")
            st = self.lib.vct_voxelize_textured(self.h, _fptr(verts), stride, verts.shape[0], _fptr(idx), idx.size,
                                                _fptr(mat) if mat is not None else None,
                                                _fptr(kd) if kd is not None else None, _fptr(mm), mm.size,
                                                uv_offset)
        self._check(st, "voxelize")

    def voxelize_device(self, verts, idx, tri_material=None, kd4=None, material_map=None, uv_offset=UV_OFFSET):
        """K1 on device-resident torch tensors: verts [V, F] float32 (F >= 3, the
        56-byte Vertex is F = 14), idx [3T] int32/uint32, tri_material [T] int32,
        kd4 [M, 4] float32, material_map [M] int32 (vct_voxelize_textured_device)."""
        if verts.dim() != 2 or verts.shape[1] < 3:
            raise VctError(_EINVAL, f"voxelize_device: verts must be [V, F >= 3], got {tuple(verts.shape)}")
        if str(idx.dtype) in _I64:
            # read as uint32 pairs, the triangles would silently collapse onto vertex 0
            raise VctError(_EINVAL, "voxelize_device: idx must be int32 / uint32, not 64-bit")
        n_idx = idx.numel()
        if n_idx % 3:
            raise VctError(_EINVAL, f"voxelize_device: {n_idx} indices, not a multiple of 3")
        if kd4 is not None and (kd4.dim() != 2 or kd4.shape[1] != 4):
            raise VctError(_EINVAL, f"voxelize_device: kd4 must be [materials, 4], got {tuple(kd4.shape)}")
        nm = 0 if kd4 is None else kd4.shape[0]
        args = (self.h, self._dev(verts, "verts"), verts.shape[1] * 4, verts.shape[0], self._dev(idx, "idx", _I32),
                n_idx, self._dev(tri_material, "tri_material", _I32, n_idx // 3), self._dev(kd4, "kd4"))
        if material_map is None:
            st = self.lib.vct_voxelize_device(*args, nm)
        else:
            # the C-ABI bounds both kd4 and the map by one n_mat: a longer map would let K1
            # read kd4 past its end on the device (the host path checks the same)
            if kd4 is not None and material_map.numel() != nm:
                raise VctError(_EINVAL, f"voxelize_device: material_map has {material_map.numel()} entries for "
                                        f"{nm} materials")
            mm = self._dev(material_map, "material_map", ("torch.int32",), max(nm, 1))
            st = self.lib.vct_voxelize_textured_device(*args, mm, material_map.numel(), uv_offset)
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
        px = width * height
        out_px = tiles_for_rank(width, height, tile_rank, tile_world) * 64 * 64 if tile_compact else px
        a.pos4 = self._dev(pos4, "pos4", _F32, 4 * px)
        a.nrm4 = self._dev(nrm4, "nrm4", _F32, 4 * px)
        a.alb4 = self._dev(alb4, "alb4", _F32, 4 * px)
        a.width, a.height = width, height
        a.eye = _f3(eye)
        a.diffuse4 = self._dev(diffuse4, "diffuse4", _F32, 4 * out_px)
        a.spec4 = self._dev(spec4, "spec4", _F32, 4 * out_px)
        a.steps_px = self._dev(steps_px, "steps_px", _I32, px)
        a.cone_steps = self._dev(cone_steps, "cone_steps", _I64, 1)
        a.texel_fetches = self._dev(texel_fetches, "texel_fetches", _I64, 1)
        a.tile_rank, a.tile_world = tile_rank, tile_world
        a.tile_compact = 1 if tile_compact else 0
        a.variant = variant
        self._check(self.lib.vct_trace_device(self.h, C.byref(a)), "trace_device")

    def untile_device(self, gathered4, width, height, world, frame4):
        g = self._dev(gathered4, "gathered4", _F32, max(world, 1) * tiles_for_rank(width, height, 0, world) * 4096 * 4)
        self._check(self.lib.vct_untile_device(self.h, g, width, height, world,
                                               self._dev(frame4, "frame4", _F32, width * height * 4)),
                    "untile_device")

    def untile_planes_device(self, gathered4, width, height, world, frames4, packed=False):
        """gathered4: [world][planes][max_tiles*64*64][4] (one all-gather of equal-size
        rank buffers) or, packed, rank r's [planes][tiles(r)*64*64][4] at tile offset
        planes * tile_offset(r) (the gather to one rank); frames4: [h][w][4] outputs."""
        planes = len(frames4)
        need = (planes * tiles_for_rank(width, height, 0, 1) if packed
                else max(world, 1) * planes * tiles_for_rank(width, height, 0, world)) * 4096 * 4
        g = self._dev(gathered4, "gathered4", _F32, need)
        arr = (C.c_void_p * planes)(*[self._dev(f, "frames4", _F32, width * height * 4) for f in frames4])
        fn = self.lib.vct_untile_planes_packed_device if packed else self.lib.vct_untile_planes_device
        self._check(fn(self.h, g, planes, width, height, world, C.cast(arr, C.c_void_p)), "untile_planes_device")

    # -- one process per GPU over RCCL (vct_comm_*) -----------
    @staticmethod
    def comm_get_id(lib=None) -> bytes:
        lib = lib if lib is not None else _lib.load()
        cid = VctCommId()
        st = lib.vct_comm_get_id(C.byref(cid))
        if st != 0:
            raise VctError(st, "vct_comm_get_id")
        return C.string_at(C.addressof(cid), 128)

    def comm_init(self, comm_id: bytes, nranks: int, rank: int):
        cid = VctCommId()
        C.memmove(C.addressof(cid), comm_id, 128)
        self._check(self.lib.vct_comm_init(self.h, C.byref(cid), nranks, rank), "comm_init")

    def comm_broadcast_level0(self, root: int = 0):
        self._check(self.lib.vct_comm_broadcast_level0(self.h, root), "comm_broadcast_level0")

    def comm_trace_frame(self, pos4, nrm4, alb4, width, height, eye, diffuse4, spec4, root=0,
                         cone_steps=None, variant=0):
        """Trace this rank's tiles and assemble the frame on `root` (VCT_ALL_RANKS: every rank)."""
        a = VctTraceArgs()
        px = width * height
        a.pos4 = self._dev(pos4, "pos4", _F32, 4 * px)
        a.nrm4 = self._dev(nrm4, "nrm4", _F32, 4 * px)
        a.alb4 = self._dev(alb4, "alb4", _F32, 4 * px)
        a.width, a.height = width, height
        a.eye = _f3(eye)
        a.diffuse4 = self._dev(diffuse4, "diffuse4", _F32, 4 * px)
        a.spec4 = self._dev(spec4, "spec4", _F32, 4 * px)
        a.cone_steps = self._dev(cone_steps, "cone_steps", _I64, 1)
        a.variant = variant
        self._check(self.lib.vct_comm_trace_frame(self.h, C.byref(a), root), "comm_trace_frame")

    def comm_destroy(self):
        self._check(self.lib.vct_comm_destroy(self.h), "comm_destroy")

    def comm_rank(self) -> tuple[int, int]:
        """(rank, nranks) of the context's communicator as RCCL holds it (vct_comm_rank;
        (0, 1) without one)."""
        r, n = C.c_uint32(), C.c_uint32()
        self._check(self.lib.vct_comm_rank(self.h, C.byref(r), C.byref(n)), "comm_rank")
        return r.value, n.value

    def comm_set_timeout(self, timeout_ms: int):
        self._check(self.lib.vct_comm_set_timeout(self.h, int(timeout_ms)), "comm_set_timeout")

    def comm_synchronize(self):
        """Wait for the queued work incl. collectives; VctError(ECOMM) after the deadline."""
        self._check(self.lib.vct_comm_synchronize(self.h), "comm_synchronize")


    def _gbuf_ptrs(self, width, height, pos4, nrm4, alb4):
        n = 4 * width * height
        return self._dev(pos4, "pos4", _F32, n), self._dev(nrm4, "nrm4", _F32, n), self._dev(alb4, "alb4", _F32, n)

    def gbuffer_raycast_device(self, cam, width, height, roughness, pos4, nrm4, alb4):
        c = cam.to_ctypes() if hasattr(cam, "to_ctypes") else cam
        self._check(self.lib.vct_gbuffer_raycast_device(self.h, C.byref(c), width, height, float(roughness),
                                                        *self._gbuf_ptrs(width, height, pos4, nrm4, alb4)),
                    "raycast")

    def gbuffer_raster_device(self, cam, width, height, roughness, pos4, nrm4, alb4):
        """Row f2: tile-binned G-buffer pass (same output as gbuffer_raycast_device)."""
        c = cam.to_ctypes() if hasattr(cam, "to_ctypes") else cam
        self._check(self.lib.vct_gbuffer_raster_device(self.h, C.byref(c), width, height, float(roughness),
                                                       *self._gbuf_ptrs(width, height, pos4, nrm4, alb4)),
                    "raster")

    def composite_device(self, pos4, nrm4, alb4, diffuse4, spec4, width, height, dir_to_light,
                         color=(1.0, 1.0, 1.0), out_linear4=None, out_rgba8=None):
        """Row f3 composite + present on device buffers (torch tensors or raw pointers)."""
        l = (C.c_float * 3)(*[float(x) for x in dir_to_light])
        c = (C.c_float * 3)(*[float(x) for x in color])
        n = 4 * width * height
        self._check(self.lib.vct_composite_device(
            self.h, *self._gbuf_ptrs(width, height, pos4, nrm4, alb4), self._dev(diffuse4, "diffuse4", _F32, n),
            self._dev(spec4, "spec4", _F32, n), width, height, l, c, self._dev(out_linear4, "out_linear4", _F32, n),
            self._dev(out_rgba8, "out_rgba8", _I32, width * height)), "composite")

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
        ptr = self._dev(dst, "dst", _F32, 4 * self.n ** 3)
        self._check(self.lib.vct_copy_level0_to_device(self.h, ptr), "copy_level0_to_device")

    def set_level0_from_device(self, src):
        ptr = self._dev(src, "src", _F32, 4 * self.n ** 3)
        self._check(self.lib.vct_set_level0_from_device(self.h, ptr), "set_level0_from_device")

    def download_voxels(self):
        n = self.n
        ao = np.empty((n, n, n, 4), np.float32)
        nm = np.empty((n, n, n, 4), np.float32)
        self._check(self.lib.vct_download_voxels(self.h, _fptr(ao), _fptr(nm)), "download_voxels")
        return ao, nm

    # -- grid dump / load (vct_save_grid / vct_load_grid; vct.dump wraps them) --------
    def save_grid(self, stem, what: int):
        """vct_save_grid: what = VCT_DUMP_* bits (vct.dump.VOXELS | LEVEL0 | PYRAMID)."""
        self._check(self.lib.vct_save_grid(self.h, os.fsencode(str(stem)), what), "save_grid")

    def load_grid(self, stem):
        """vct_load_grid: replaces this context's grid state with the dump's."""
        self._check(self.lib.vct_load_grid(self.h, os.fsencode(str(stem))), "load_grid")

    def download_accum(self):
        n = self.n
        sums = np.empty((n ** 3, 6), np.int64)
        counts = np.empty((n ** 3,), np.uint32)
        self._check(self.lib.vct_download_accum(self.h, _fptr(sums), _fptr(counts)), "download_accum")
        return sums, counts


def comm_frame_layout(w: int, h: int, nranks: int, rank: int, root: int, lib=None) -> dict:
    """vct_comm_frame_layout: where rank's tiles sit in the frame exchange buffer."""
    from ._lib import VctCommLayout
    lib = lib if lib is not None else _lib.load()
    out = VctCommLayout()
    st = lib.vct_comm_frame_layout(w, h, nranks, rank, root, C.byref(out))
    if st != 0:
        raise VctError(st, "vct_comm_frame_layout")
    return {f: int(getattr(out, f)) for f, _ in VctCommLayout._fields_}
