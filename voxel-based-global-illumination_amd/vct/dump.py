"""Grid and G-buffer dump / load: raw ``.bin`` + JSON header (SURVEY.md §5 "checkpoint /
resume": golden fixtures and repro cases; the reference persists no state).

A dump is two files: ``<stem>.json`` (what the data is) and ``<stem>.bin`` (little-endian
float32, C order).

* **Grid** (:func:`save_grid` / :func:`load_grid`). The header holds the context config
  (n, aabb_min, extent, aniso, cone set) and the byte length and sha256 of the payload.
  The payload is level 0 as [z][y][x][rgba], the linear layout of ``vct_download_level``
  and ``vct_upload_level0``. With ``pyramid=True`` it also holds every face of levels
  1..L, in level-major then face-major order.
  - Loading uploads level 0 and runs ``vct_build_mips``, which is deterministic.
  - The rebuilt pyramid is therefore bit-identical to the dumped one. When the dump
    carries the pyramid, ``verify=True`` checks that.
* **G-buffer** (:func:`save_gbuffer` / :func:`load_gbuffer`). ``pos4`` / ``nrm4`` /
  ``alb4`` are [h][w][4] float32 (vct_trace_args), plus the eye position.

The payload is checked against the header's length and sha256 before anything is
uploaded. A truncated or edited dump raises ``ValueError``.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

FORMAT = "vct-dump/1"


def _paths(stem: str):
    stem = str(stem)
    if stem.endswith(".json") or stem.endswith(".bin"):
        stem = stem.rsplit(".", 1)[0]
    return stem + ".json", stem + ".bin"


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
    header = dict(header, format=FORMAT, payload=os.path.basename(bpath), bytes=size, sha256=h.hexdigest())
    with open(jpath, "w") as f:
        json.dump(header, f, indent=1, sort_keys=True)


def _read(stem: str, kind: str):
    jpath, bpath = _paths(stem)
    with open(jpath) as f:
        header = json.load(f)
    if header.get("format") != FORMAT or header.get("kind") != kind:
        raise ValueError(f"{jpath}: not a {FORMAT} {kind} dump")
    with open(bpath, "rb") as f:
        raw = f.read()
    if len(raw) != header["bytes"] or hashlib.sha256(raw).hexdigest() != header["sha256"]:
        raise ValueError(f"{bpath}: payload does not match its header (length or sha256)")
    return header, np.frombuffer(raw, dtype="<f4")


def save_grid(ctx, stem: str, pyramid: bool = False) -> None:
    """Dump ctx's level 0 (and, pyramid=True, every face of levels 1..L)."""
    arrays = [ctx.download_level(0)]
    levels = []
    for l in range(ctx.num_levels):
        nl, nf = ctx.level_dims(l)
        levels.append({"level": l, "n": int(nl), "faces": int(nf)})
        if pyramid and l > 0:
            arrays += [ctx.download_level(l, f) for f in range(nf)]
    header = {"kind": "grid", "n": ctx.n, "aabb_min": list(ctx.aabb_min), "extent": ctx.extent,
              "aniso": bool(ctx.aniso), "n_diffuse": ctx.n_diffuse, "specular": bool(ctx.specular),
              "levels": levels, "pyramid": bool(pyramid)}
    _write(stem, header, arrays)


def load_grid(stem: str, ctx=None, verify: bool = True, **ctx_kw):
    """Context (new, or ctx with the same n / aniso) holding the dumped grid: level 0
    uploaded, mips rebuilt; with a dumped pyramid and verify, checked bit for bit."""
    from . import Context
    header, data = _read(stem, "grid")
    n = int(header["n"])
    if ctx is None:
        ctx = Context(n, header["aabb_min"], header["extent"], aniso=header["aniso"],
                      n_diffuse=header["n_diffuse"], specular=header["specular"], **ctx_kw)
    elif ctx.n != n or bool(ctx.aniso) != bool(header["aniso"]):
        raise ValueError(f"dump is n={n} aniso={header['aniso']}, context n={ctx.n} aniso={ctx.aniso}")
    nv = n ** 3 * 4
    if data.size < nv:
        raise ValueError("payload shorter than level 0")
    ctx.upload_level0(data[:nv].reshape(n, n, n, 4))
    ctx.build_mips()
    if header["pyramid"] and verify:
        off = nv
        for lv in header["levels"][1:]:
            cnt = lv["n"] ** 3 * 4
            for f in range(lv["faces"]):
                want = data[off:off + cnt].reshape(lv["n"], lv["n"], lv["n"], 4)
                if not np.array_equal(ctx.download_level(lv["level"], f), want):
                    raise ValueError(f"rebuilt level {lv['level']} face {f} differs from the dump")
                off += cnt
    return ctx


def save_gbuffer(stem: str, pos4: np.ndarray, nrm4: np.ndarray, alb4: np.ndarray, eye) -> None:
    h, w = pos4.shape[:2]
    for a in (pos4, nrm4, alb4):
        if a.shape != (h, w, 4):
            raise ValueError(f"G-buffer planes must be [h][w][4], got {a.shape}")
    _write(stem, {"kind": "gbuffer", "width": int(w), "height": int(h), "eye": [float(x) for x in eye]},
           [pos4, nrm4, alb4])


def load_gbuffer(stem: str):
    """-> (pos4, nrm4, alb4, eye) as [h][w][4] float32 arrays and a 3-tuple"""
    header, data = _read(stem, "gbuffer")
    w, h = int(header["width"]), int(header["height"])
    if data.size != 3 * h * w * 4:
        raise ValueError("G-buffer payload size does not match width x height")
    planes = data.reshape(3, h, w, 4).copy()
    return planes[0], planes[1], planes[2], tuple(header["eye"])
