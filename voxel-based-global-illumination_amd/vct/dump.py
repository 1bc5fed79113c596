"""Grid and G-buffer dump / load (SURVEY.md §5 "checkpoint / resume": golden fixtures,
repro cases, relighting a saved scene; the reference persists no state).

* **Grid** (:func:`save_grid` / :func:`load_grid`) is the C-ABI's ``vct_save_grid`` /
  ``vct_load_grid`` (``include/vct.h``), so the C++ host and Python write the same files
  (format ``vct-dump/2``, spelled out in ``csrc/vct_dumpio.h``): ``<stem>.json`` (grid
  config, sections, payload length and sha256) + ``<stem>.bin``. Sections:

  - ``VOXELS``: K1's state, the occupied voxels' integer sums and counts. A context loaded
    from it is voxelized: any light can be injected, the mips built, frames traced and
    composited, bit for bit as after the original ``vct_voxelize`` (the triangles are not
    dumped);
  - ``LEVEL0``: the level-0 radiance; loading it builds the mips at once;
  - ``PYRAMID``: every face of levels 1..L; the rebuilt pyramid is checked against it bit
    for bit on load.

  Loading checks the payload's length and sha256 and that the dump's grid (n, aabb_min,
  extent, aniso) is the context's before anything changes; a mismatch or a damaged dump
  raises ``ValueError``.
* **G-buffer** (:func:`save_gbuffer` / :func:`load_gbuffer`, Python only: the planes are the
  host's own data). ``pos4`` / ``nrm4`` / ``alb4`` are [h][w][4] float32 (vct_trace_args),
  plus the eye position; ``<stem>.json`` + ``<stem>.bin`` (format ``vct-dump/1``, kind
  ``gbuffer``), the payload checked against the header's length and sha256.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os

import numpy as np

from . import _lib

VOXELS, LEVEL0, PYRAMID = 0x1, 0x2, 0x4   # VCT_DUMP_*
GBUF_FORMAT = "vct-dump/1"
_EINVAL = 1


def _paths(stem: str):
    stem = str(stem)
    if stem.endswith(".json") or stem.endswith(".bin"):
        stem = stem.rsplit(".", 1)[0]
    return stem + ".json", stem + ".bin"


def dump_info(stem, lib=None):
    """(vct_config fields as a dict, what) of a grid dump's header (vct_dump_info)."""
    lib = lib if lib is not None else _lib.load()
    cfg, what = _lib.VctConfig(), C.c_uint32()
    if lib.vct_dump_info(os.fsencode(_paths(stem)[0]), C.byref(cfg), C.byref(what)) != 0:
        raise ValueError(f"{_paths(stem)[0]}: not a readable vct-dump/2 grid header")
    return {"n": cfg.n, "aabb_min": tuple(cfg.aabb_min), "extent": cfg.extent, "aniso": bool(cfg.aniso),
            "n_diffuse": cfg.n_diffuse, "specular": bool(cfg.specular)}, what.value


def save_grid(ctx, stem, pyramid: bool = False, voxels: bool = True, level0: bool = True) -> None:
    """Dump ctx's K1 state (voxels), level 0 and, pyramid=True, every face of levels 1..L."""
    what = (VOXELS if voxels else 0) | (LEVEL0 if level0 else 0) | (PYRAMID if pyramid else 0)
    ctx.save_grid(_paths(stem)[0], what)


def load_grid(stem, ctx=None, verify: bool = True, **ctx_kw):
    """A context (new, or ctx of the same grid) holding the dumped state.  A dumped pyramid
    is always verified against the rebuilt one (verify is kept for callers' clarity)."""
    from . import Context, VctError
    del verify
    info, _ = dump_info(stem, lib=ctx.lib if ctx is not None else ctx_kw.get("lib"))
    if ctx is None:
        ctx = Context(info["n"], info["aabb_min"], info["extent"], aniso=info["aniso"],
                      n_diffuse=info["n_diffuse"], specular=info["specular"], **ctx_kw)
    try:
        ctx.load_grid(_paths(stem)[0])
    except VctError as e:
        if e.status == _EINVAL:
            raise ValueError(str(e)) from None
        raise
    return ctx


def _write(stem: str, header: dict, arrays) -> None:
    jpath, bpath = _paths(stem)
    h = hashlib.sha256()
    size = 0
    with open(bpath, "wb") as f:
        for a in arrays:
            b = np.ascontiguousarray(a, dtype="<f4").tobytes()
            h.update(b)
            size += len(b)
            f.write(b)
    header = dict(header, format=GBUF_FORMAT, payload=os.path.basename(bpath), bytes=size, sha256=h.hexdigest())
    with open(jpath, "w") as f:
        json.dump(header, f, indent=1, sort_keys=True)


def _read(stem: str, kind: str):
    jpath, bpath = _paths(stem)
    with open(jpath) as f:
        header = json.load(f)
    if header.get("format") != GBUF_FORMAT or header.get("kind") != kind:
        raise ValueError(f"{jpath}: not a {GBUF_FORMAT} {kind} dump")
    with open(bpath, "rb") as f:
        raw = f.read()
    if len(raw) != header["bytes"] or hashlib.sha256(raw).hexdigest() != header["sha256"]:
        raise ValueError(f"{bpath}: payload does not match its header (length or sha256)")
    return header, np.frombuffer(raw, dtype="<f4")


def save_gbuffer(stem, pos4: np.ndarray, nrm4: np.ndarray, alb4: np.ndarray, eye) -> None:
    h, w = pos4.shape[:2]
    for a in (pos4, nrm4, alb4):
        if a.shape != (h, w, 4):
            raise ValueError(f"G-buffer planes must be [h][w][4], got {a.shape}")
    _write(stem, {"kind": "gbuffer", "width": int(w), "height": int(h), "eye": [float(x) for x in eye]},
           [pos4, nrm4, alb4])


def load_gbuffer(stem):
    """-> (pos4, nrm4, alb4, eye) as [h][w][4] float32 arrays and a 3-tuple"""
    header, data = _read(stem, "gbuffer")
    w, h = int(header["width"]), int(header["height"])
    if data.size != 3 * h * w * 4:
        raise ValueError("G-buffer payload size does not match width x height")
    planes = data.reshape(3, h, w, 4).copy()
    return planes[0], planes[1], planes[2], tuple(header["eye"])
