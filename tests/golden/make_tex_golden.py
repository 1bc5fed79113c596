"""Texture fixtures for the diffuse-map row (SURVEY 8a Model::loadMaterials).

Run in the build container (it needs /root/reference and oracle/_ref/ref_stb_probe,
the reference's own stb_image compiled by `make -C oracle ref`):

    python tests/golden/make_tex_golden.py

Writes tests/golden/tex_png_cases.npz and tests/golden/tex_nanosuit.npz:

* tex_png_cases.npz -- PNG files this script writes itself (every colour type, bit
  depth 1..16, tRNS keys and palette alpha, Adam7 interlacing, all five scanline
  filters, split IDAT, an ancillary chunk), each with what the reference's
  stbi_load(.., 0) (assets/code/scene/model.cpp:197) returned for it: the pins of
  the host PNG decoder (host/png.cpp).  Keys: case names, png_<name> (file bytes),
  stb_<name> (h x w x comp uint8, or an empty array when stb refused the file).
* tex_nanosuit.npz -- the reference's own texture files (assets/model/test/*.png):
  per file the stbi_load size / channel count and the sha256 of its pixel bytes
  (checked against host/png.cpp when /root/reference is present), and for the six
  diffuse maps nanosuit.mtl names (map_Kd, nanosuit.mtl:11,24,37,49,62,74) a 64x64
  RGBA8 crop (channels expanded as the GL upload samples them), the textures of the
  GPU parity test.  The crops are data taken from those files; no source is stored.
"""
from __future__ import annotations

import hashlib
import os
import struct
import subprocess
import sys
import tempfile
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PROBE = os.path.join(REPO, "oracle", "_ref", "ref_stb_probe")
REF_TEX = "/root/reference/assets/model/test"
DIFFUSE_MAPS = ["arm_dif.png", "body_dif.png", "glass_dif.png", "hand_dif.png", "helmet_diff.png", "leg_dif.png"]
CROP = 64


# ---------------------------------------------------------------------------
# a small PNG writer (any colour type / depth / interlace / filter choice)
# ---------------------------------------------------------------------------
def _chunk(t: bytes, d: bytes) -> bytes:
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def _filter_row(raw: bytes, prev: bytes, ft: int, bpp: int) -> bytes:
    out = bytearray([ft])
    for i, x in enumerate(raw):
        a = raw[i - bpp] if i >= bpp else 0
        b = prev[i]
        c = prev[i - bpp] if i >= bpp else 0
        pred = (0, a, b, (a + b) >> 1, _paeth(a, b, c))[ft]
        out.append((x - pred) & 255)
    return bytes(out)


def _pack_row(samples: np.ndarray, depth: int) -> bytes:
    """samples: (w, ch) ints -> the scanline bytes at this depth"""
    flat = samples.reshape(-1).astype(np.int64)
    if depth == 16:
        return b"".join(struct.pack(">H", int(v)) for v in flat)
    if depth == 8:
        return bytes(int(v) for v in flat)
    out, acc, nb = bytearray(), 0, 0
    for v in flat:
        acc = (acc << depth) | int(v)
        nb += depth
        if nb == 8:
            out.append(acc)
            acc, nb = 0, 0
    if nb:
        out.append(acc << (8 - nb))
    return bytes(out)


def write_png(img: np.ndarray, color: int, depth: int, interlace=False, plte=None, trns=None, filters=None,
              split_idat=False, extra=True) -> bytes:
    """img: (h, w, ch) sample values at `depth` (palette: indices)."""
    h, w, ch = img.shape
    rng = np.random.default_rng(h * 131 + w * 7 + depth + color)
    bpp = max(1, ch * depth // 8)
    passes = ([(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]
              if interlace else [(0, 0, 1, 1)])
    raw = bytearray()
    for xo, yo, xs, ys in passes:
        sub = img[yo::ys, xo::xs]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        prev = bytes(len(_pack_row(sub[0], depth)))
        for y in range(sub.shape[0]):
            row = _pack_row(sub[y], depth)
            ft = int(rng.integers(0, 5)) if filters is None else filters[y % len(filters)]
            raw += _filter_row(row, prev, ft, bpp)
            prev = row
    z = zlib.compress(bytes(raw), 9)
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, color, 0, 0, int(interlace)))
    if extra:
        out += _chunk(b"tEXt", b"Comment\x00fixture")
    if plte is not None:
        out += _chunk(b"PLTE", bytes(np.asarray(plte, np.uint8).reshape(-1)))
    if trns is not None:
        out += _chunk(b"tRNS", trns)
    if split_idat:
        k = max(1, len(z) // 3)
        for i in range(0, len(z), k):
            out += _chunk(b"IDAT", z[i:i + k])
    else:
        out += _chunk(b"IDAT", z)
    return out + _chunk(b"IEND", b"")


def png_cases():
    rng = np.random.default_rng(2024)
    cases = {}
    chans = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}
    for color, depths in ((0, (1, 2, 4, 8, 16)), (2, (8, 16)), (3, (1, 2, 4, 8)), (4, (8, 16)), (6, (8, 16))):
        for depth in depths:
            for (w, h) in ((13, 7), (1, 1), (9, 17)):
                for il in (False, True):
                    top = (1 << depth) - 1
                    plte = trns = None
                    if color == 3:
                        npal = min(1 << depth, 40)
                        top = npal - 1
                        plte = rng.integers(0, 256, (npal, 3))
                    img = rng.integers(0, top + 1, (h, w, chans[color]))
                    name = f"c{color}_d{depth}_{w}x{h}{'_i' if il else ''}"
                    cases[name] = write_png(img, color, depth, il, plte=plte, split_idat=(w == 9))
                    # tRNS variants: a colour key that some pixels hit / palette alpha
                    if color in (0, 2) and w == 13:
                        key = img[0, 0]
                        tr = b"".join(struct.pack(">H", int(v)) for v in key)
                        cases[name + "_trns"] = write_png(img, color, depth, il, trns=tr)
                    if color == 3 and w == 13:
                        alpha = bytes(int(v) for v in rng.integers(0, 256, max(1, len(plte) // 2)))
                        cases[name + "_trns"] = write_png(img, color, depth, il, plte=plte, trns=alpha)
    # one case per single filter type (RGBA 8)
    img = rng.integers(0, 256, (11, 10, 4))
    for ft in range(5):
        cases[f"rgba_filter{ft}"] = write_png(img, 6, 8, filters=[ft], extra=False)
    # headers that declare a huge image over a few bytes of data: stb refuses the first
    # two as too large (2^30 / w / channels < h; a palette image counts 4 channels), the
    # third is at the limit and fails for want of pixels -- none may size a buffer from
    # the header alone (host/png.cpp)
    for name, (w, h, color, plte) in {"huge_rgba": (1 << 15, 1 << 15, 6, None),
                                      "huge_pal": (1 << 14, 1 << 15, 3, [[1, 2, 3]]),
                                      "limit_gray": (1 << 15, 1 << 15, 0, None)}.items():
        out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, color, 0, 0, 0))
        if plte is not None:
            out += _chunk(b"PLTE", bytes(np.asarray(plte, np.uint8).reshape(-1)))
        cases[name] = out + _chunk(b"IDAT", zlib.compress(bytes(64), 9)) + _chunk(b"IEND", b"")
    return cases


def run_probe(files):
    """-> list of (w, h, comp, bytes) or None per file, via the reference's stb_image"""
    with tempfile.TemporaryDirectory() as d:
        args, outs = [], []
        for i, f in enumerate(files):
            o = os.path.join(d, f"{i}.raw")
            args += [f, o]
            outs.append(o)
        res = subprocess.run([PROBE] + args, capture_output=True, text=True, check=True).stdout.splitlines()
        got = []
        for line, o in zip(res, outs):
            if line.startswith("fail"):
                got.append(None)
                continue
            w, h, c = (int(x) for x in line.split())
            got.append((w, h, c, open(o, "rb").read()))
        return got


def expand_rgba(data: np.ndarray) -> np.ndarray:
    """GL_RED / GL_RGB / GL_RGBA upload as sampled (vct_spec.h diffuse maps)"""
    h, w, c = data.shape
    out = np.zeros((h, w, 4), np.uint8)
    out[..., 3] = 255
    if c == 1:
        out[..., 0] = data[..., 0]
    elif c in (3, 4):
        out[..., :c] = data
    else:
        raise ValueError("2-channel texture")
    return out


def main():
    if not os.path.exists(PROBE):
        sys.exit(f"{PROBE} missing: run `make -C oracle ref` in the build container")
    cases = png_cases()
    with tempfile.TemporaryDirectory() as d:
        paths = []
        for name, blob in cases.items():
            p = os.path.join(d, name + ".png")
            open(p, "wb").write(blob)
            paths.append(p)
        decoded = run_probe(paths)
    out = {"names": np.array(list(cases.keys()))}
    for (name, blob), got in zip(cases.items(), decoded):
        out["png_" + name] = np.frombuffer(blob, np.uint8)
        if got is None:
            out["stb_" + name] = np.zeros((0,), np.uint8)
        else:
            w, h, c, raw = got
            out["stb_" + name] = np.frombuffer(raw, np.uint8).reshape(h, w, c)
    np.savez_compressed(os.path.join(HERE, "tex_png_cases.npz"), **out)
    print("png cases:", len(cases))

    files = sorted(f for f in os.listdir(REF_TEX) if f.endswith(".png"))
    decoded = run_probe([os.path.join(REF_TEX, f) for f in files])
    ref = {"files": np.array(files), "maps": np.array(DIFFUSE_MAPS)}
    meta = []
    for f, got in zip(files, decoded):
        w, h, c, raw = got
        meta.append((w, h, c))
        ref["sha256_" + f] = np.frombuffer(hashlib.sha256(raw).digest(), np.uint8)
        if f in DIFFUSE_MAPS:
            img = expand_rgba(np.frombuffer(raw, np.uint8).reshape(h, w, c))
            y0, x0 = (h - CROP) // 2 - h // 8, (w - CROP) // 2 + w // 16
            ref["crop_" + f] = np.ascontiguousarray(img[y0:y0 + CROP, x0:x0 + CROP])
            ref["crop_at_" + f] = np.array([y0, x0])
    ref["whc"] = np.array(meta, np.int64)
    np.savez_compressed(os.path.join(HERE, "tex_nanosuit.npz"), **ref)
    print("reference textures:", len(files), "diffuse crops:", len(DIFFUSE_MAPS))


if __name__ == "__main__":
    main()
