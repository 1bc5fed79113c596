"""Diffuse maps (SURVEY 8a Model::loadMaterials: albedo = Kd x diffuse map), CPU side.

* host PNG decoder (host/png.cpp) == the reference's own stb_image
  (assets/code/support/stb_image.cpp compiled by oracle/Makefile `ref`): every
  colour type / bit depth / tRNS / interlace / filter case of
  tests/golden/tex_png_cases.npz, and -- where /root/reference exists -- the
  reference's 17 texture files by sha256 (tests/golden/tex_nanosuit.npz);
* the loader's map_Kd handling (loadMaterialTextures, model.cpp:150-186): shared
  per path, channel expansion as GL_RED / GL_RGB sample, failures reported;
* the sampling rule of vct_spec.h pinned by closed forms (texel centres, repeat,
  bilinear midpoints, barycentric clamping) and by the independent restatement
  tests/spec_ref.py (textured K1 bit for bit);
* the CPU backend of include/vct.h: vct_set_textures / vct_voxelize_textured state
  and error codes, and the G-buffer albedo at the hit UV.
"""
import ctypes as C
import hashlib
import os
import subprocess

import numpy as np
import pytest

import spec_ref as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "voxel-based-global-illumination_amd")
HOST_LIB = os.path.join(PKG, "vct", "libvct_host.so")
GOLD = os.path.join(REPO, "tests", "golden")
REF_TEX = "/root/reference/assets/model/test"


@pytest.fixture(scope="module")
def host():
    if not os.path.exists(HOST_LIB):
        subprocess.run(["make", "-C", PKG, "vct/libvct_host.so"], check=True, capture_output=True)
    lib = C.CDLL(HOST_LIB)
    P = C.c_void_p
    lib.vcth_decode_png.argtypes = [P, C.c_size_t, C.POINTER(P), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                    C.POINTER(C.c_int), C.c_char_p, C.c_int]
    lib.vcth_free_image.argtypes = [P]
    lib.vcth_load_obj.argtypes = [C.c_char_p, C.POINTER(P), C.c_char_p, C.c_int]
    lib.vcth_num_materials.argtypes = [P]
    lib.vcth_num_materials.restype = C.c_uint32
    lib.vcth_num_textures.argtypes = [P]
    lib.vcth_num_textures.restype = C.c_uint32
    lib.vcth_texture.argtypes = [P, C.c_uint32, C.POINTER(P), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_char_p)]
    lib.vcth_material_diffuse_map.argtypes = [P, C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_int32)]
    lib.vcth_num_texture_errors.argtypes = [P]
    lib.vcth_num_texture_errors.restype = C.c_uint32
    lib.vcth_texture_error.argtypes = [P, C.c_uint32]
    lib.vcth_texture_error.restype = C.c_char_p
    lib.vcth_free.argtypes = [P]
    return lib


def decode(lib, blob: bytes):
    buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
    data, w, h, comp = C.c_void_p(), C.c_uint32(), C.c_uint32(), C.c_int()
    err = C.create_string_buffer(128)
    if lib.vcth_decode_png(C.cast(buf, C.c_void_p), len(blob), C.byref(data), C.byref(w), C.byref(h), C.byref(comp),
                           err, 128) != 0:
        return None, err.value.decode()
    n = w.value * h.value * comp.value
    out = np.ctypeslib.as_array(C.cast(data, C.POINTER(C.c_uint8)), (n,)).copy().reshape(h.value, w.value, comp.value)
    lib.vcth_free_image(data)
    return out, ""


# ---------------------------------------------------------------------------
# PNG decoder vs the reference's stb_image
# ---------------------------------------------------------------------------
def test_png_decoder_matches_reference_stb(host):
    g = np.load(os.path.join(GOLD, "tex_png_cases.npz"))
    names = list(g["names"])
    assert len(names) > 100
    refused = 0
    for name in names:
        got, err = decode(host, g["png_" + name].tobytes())
        ref = g["stb_" + name]
        if not ref.size:           # stb refused the file (the huge-header cases): so must we
            assert got is None, name
            refused += 1
            continue
        assert got is not None, (name, err)
        assert got.shape == ref.shape, (name, got.shape, ref.shape)
        assert np.array_equal(got, ref), name
    assert refused == 3       # huge_rgba, huge_pal (stb: "too large"), limit_gray (not enough pixels)


def test_png_decoder_refuses_corrupt_files(host):
    g = np.load(os.path.join(GOLD, "tex_png_cases.npz"))
    good = g["png_c6_d8_13x7"].tobytes()
    assert decode(host, good)[0] is not None
    assert decode(host, b"GIF89a" + good[6:])[0] is None                 # signature
    assert decode(host, good[:60])[0] is None                             # truncated inside IDAT
    bad_ihdr = bytearray(good)
    bad_ihdr[24] = 3                                                      # bit depth 3
    assert "depth" in decode(host, bytes(bad_ihdr))[1]
    # a header declaring more than stb's 2^30-byte limit (stb_image.h:4837-4845) is refused
    # before anything is sized from it; so is one within the limit over too little data
    assert "too large" in decode(host, g["png_huge_rgba"].tobytes())[1]
    assert "too large" in decode(host, g["png_huge_pal"].tobytes())[1]
    assert "not enough pixels" in decode(host, g["png_limit_gray"].tobytes())[1]


@pytest.mark.skipif(not os.path.isdir(REF_TEX), reason="the reference's texture files exist only in the build container")
def test_png_decoder_on_reference_textures(host):
    """All 17 PNGs the reference ships decode to the bytes its stb_image returns."""
    r = np.load(os.path.join(GOLD, "tex_nanosuit.npz"))
    for f, (w, h, c) in zip(r["files"], r["whc"]):
        got, err = decode(host, open(os.path.join(REF_TEX, str(f)), "rb").read())
        assert got is not None, (f, err)
        assert got.shape == (h, w, c), f
        assert hashlib.sha256(got.tobytes()).digest() == r["sha256_" + str(f)].tobytes(), f


# ---------------------------------------------------------------------------
# loader: map_Kd -> textures (loadMaterialTextures / TextureFromFile)
# ---------------------------------------------------------------------------
def _png(img, color):
    import importlib.util
    spec = importlib.util.spec_from_file_location("mtg", os.path.join(GOLD, "make_tex_golden.py"))
    mtg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mtg)
    return mtg.write_png(img, color, 8)


def test_loader_loads_and_shares_diffuse_maps(host, tmp_path):
    rng = np.random.default_rng(3)
    rgba = rng.integers(0, 256, (5, 6, 4))
    grey = rng.integers(0, 256, (4, 3, 1))
    rgb = rng.integers(0, 256, (3, 7, 3))
    ga = rng.integers(0, 256, (2, 2, 2))
    (tmp_path / "rgba.png").write_bytes(_png(rgba, 6))
    (tmp_path / "grey.png").write_bytes(_png(grey, 0))
    (tmp_path / "rgb.png").write_bytes(_png(rgb, 2))
    (tmp_path / "ga.png").write_bytes(_png(ga, 4))
    (tmp_path / "scene.mtl").write_text(
        "newmtl a\nKd 1 1 1\nmap_Kd rgba.png\n"
        "newmtl b\nKd 0.5 0.5 0.5\nmap_Kd -clamp on grey.png\n"
        "newmtl c\nKd 1 0 0\nmap_Kd rgba.png\n"            # same path as a: shared texture
        "newmtl d\nKd 0 1 0\nmap_Kd rgb.png\n"
        "newmtl e\nKd 0 0 1\nmap_Kd ga.png\n"              # 2 channels: refused
        "newmtl f\nKd 1 1 0\nmap_Kd missing.png\n"         # missing: refused
        "newmtl g\nKd 1 1 1\n")
    (tmp_path / "m.obj").write_text("mtllib scene.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nvt 0 0\n"
                                    "usemtl a\nf 1/1/1 2/1/1 3/1/1\n")
    h = C.c_void_p()
    err = C.create_string_buffer(256)
    assert host.vcth_load_obj(str(tmp_path / "m.obj").encode(), C.byref(h), err, 256) == 0
    maps = {}
    for i in range(host.vcth_num_materials(h)):
        p, t = C.c_char_p(), C.c_int32()
        host.vcth_material_diffuse_map(h, i, C.byref(p), C.byref(t))
        maps[i] = (p.value.decode(), t.value)
    # DefaultMaterial first, then a..g
    assert maps[0] == ("", -1)
    assert maps[1] == ("rgba.png", 0) and maps[3] == ("rgba.png", 0)
    assert maps[2] == ("grey.png", 1) and maps[4] == ("rgb.png", 2)
    assert maps[5] == ("ga.png", -1) and maps[6] == ("missing.png", -1) and maps[7] == ("", -1)
    assert host.vcth_num_textures(h) == 3
    errs = [host.vcth_texture_error(h, i).decode() for i in range(host.vcth_num_texture_errors(h))]
    assert any("ga.png" in e and "2-channel" in e for e in errs) and any("missing.png" in e for e in errs)
    expect = []
    for src, comp in ((rgba, 4), (grey, 1), (rgb, 3)):
        e = np.zeros(src.shape[:2] + (4,), np.uint8)
        e[..., 3] = 255
        if comp == 1:
            e[..., 0] = src[..., 0]          # GL_RED samples (r, 0, 0, 1)
        else:
            e[..., :comp] = src
        expect.append(e)
    for i, e in enumerate(expect):
        d, w, hh, p = C.c_void_p(), C.c_uint32(), C.c_uint32(), C.c_char_p()
        assert host.vcth_texture(h, i, C.byref(d), C.byref(w), C.byref(hh), C.byref(p)) == 0
        got = np.ctypeslib.as_array(C.cast(d, C.POINTER(C.c_uint8)), (hh.value * w.value * 4,))
        assert np.array_equal(got.reshape(hh.value, w.value, 4), e), i
    host.vcth_free(h)


# ---------------------------------------------------------------------------
# sampling rule: closed forms on the oracle
# ---------------------------------------------------------------------------
def test_tex_sample_known_answers(oracle_mod):
    O = oracle_mod
    rng = np.random.default_rng(5)
    t = rng.integers(0, 256, (6, 8, 4)).astype(np.uint8)
    H, W = t.shape[:2]
    # texel centres return the texel exactly (c / 255)
    for y in range(H):
        for x in range(W):
            got = O.tex_sample(t, (x + 0.5) / W, (y + 0.5) / H)
            assert np.array_equal(got, t[y, x, :3].astype(np.float32) / np.float32(255)), (x, y)
    # GL_REPEAT: whole-number shifts of the coordinate change nothing (exact for these values)
    for u, v in ((0.3125, 0.25), (0.0625, 0.75)):
        a = O.tex_sample(t, u, v)
        for du, dv in ((1, 0), (-2, 0), (0, 3), (-1, -1)):
            assert np.array_equal(O.tex_sample(t, u + du, v + dv), a)
    # the wrap seam: u = 0 is half way between the last and the first column
    got = O.tex_sample(t, 0.0, 0.5 / H)
    c0, cl = t[0, 0, :3].astype(np.float32) / 255, t[0, W - 1, :3].astype(np.float32) / 255
    assert np.allclose(got, (c0 + cl) / 2, atol=1e-6)
    # a constant texture samples its value everywhere; non-finite coordinates read as 0
    k = np.full((3, 5, 4), 200, np.uint8)
    for u, v in ((0.123, 0.877), (-7.4, 19.2), (np.inf, 0.5), (np.nan, np.nan)):
        assert np.array_equal(O.tex_sample(k, u, v), np.full(3, np.float32(200) / np.float32(255)))
    assert np.array_equal(O.tex_sample(t, np.nan, np.inf), O.tex_sample(t, 0.0, 0.0))


def test_tri_bary_known_answers(oracle_mod):
    O = oracle_mod
    q0, q1, q2 = (0, 0, 0), (4, 0, 0), (0, 4, 0)
    assert O.tri_bary(q0, q1, q2, (0, 0, 0)) == (0.0, 0.0)
    assert O.tri_bary(q0, q1, q2, (4, 0, 0)) == (1.0, 0.0)
    assert O.tri_bary(q0, q1, q2, (0, 4, 2.5)) == (0.0, 1.0)           # off the plane: projected
    assert O.tri_bary(q0, q1, q2, (1, 2, -3)) == (0.25, 0.5)
    assert O.tri_bary(q0, q1, q2, (-3, -1, 0)) == (0.0, 0.0)           # clamped into the triangle
    b1, b2 = O.tri_bary(q0, q1, q2, (8, 8, 0))                         # beyond the hypotenuse
    assert (b1, b2) == (0.5, 0.5)
    assert O.tri_bary(q0, q0, q0, (1, 1, 1)) == (0.0, 0.0)             # degenerate -> vertex 0
    assert O.tri_uv((0.5, 0.25, 2.5, 0.25, 0.5, -1.75), 0.25, 0.5) == (1.0, -0.75)


# ---------------------------------------------------------------------------
# textured K1: C oracle == the independent restatement, bit for bit
# ---------------------------------------------------------------------------
def _textured_case(seed, n=16, n_tri=24):
    rng = np.random.default_rng(seed)
    verts = np.zeros((3 * n_tri, 14), np.float32)
    c = rng.uniform(-0.8, 0.8, (n_tri, 3))
    verts[:, :3] = (c[:, None, :] + rng.uniform(-0.35, 0.35, (n_tri, 3, 3))).reshape(-1, 3)
    verts[:, 6:8] = rng.uniform(-1.5, 2.5, (3 * n_tri, 2))
    idx = np.arange(3 * n_tri, dtype=np.uint32)
    tri_mat = rng.integers(0, 4, n_tri).astype(np.uint32)
    kd = rng.uniform(0.2, 1.0, (4, 4)).astype(np.float32)
    textures = [rng.integers(0, 256, (5, 7, 4)).astype(np.uint8), rng.integers(0, 256, (9, 4, 4)).astype(np.uint8)]
    mat_map = np.array([0, -1, 1, 0], np.int32)
    g0, E = (-1.0, -1.0, -1.0), 2.0
    return n, g0, E, verts, idx, tri_mat, kd, mat_map, textures


@pytest.mark.parametrize("seed", [1, 2])
def test_textured_voxelize_oracle_equals_spec_ref(oracle_mod, seed):
    n, g0, E, verts, idx, tri_mat, kd, mat_map, textures = _textured_case(seed)
    sums, counts = oracle_mod.voxelize(n, g0, E, verts, idx, tri_mat, kd, mat_map, textures)
    rs, rc = S.voxelize(n, g0, E, verts, idx, tri_mat, kd, mat_map=mat_map, textures=textures)
    assert np.array_equal(counts, rc)
    assert np.array_equal(sums, rs)
    # the untextured rule is the mat_map = -1 case
    s0, c0 = oracle_mod.voxelize(n, g0, E, verts, idx, tri_mat, kd)
    s1, c1 = oracle_mod.voxelize(n, g0, E, verts, idx, tri_mat, kd, np.full(4, -1, np.int32), textures)
    assert np.array_equal(s0, s1) and np.array_equal(c0, c1)


def test_textured_voxelize_constant_map_is_kd_times_value(oracle_mod):
    """A constant-colour map scales Kd: albedo = Kd * c/255 in every voxel it covers."""
    n, g0, E, verts, idx, tri_mat, kd, _, _ = _textured_case(4)
    tex = [np.full((3, 3, 4), (51, 102, 255, 255), np.uint8)]
    kd[:] = (0.5, 0.75, 1.0, 1.0)
    sums, counts = oracle_mod.voxelize(n, g0, E, verts, idx, tri_mat, kd, np.zeros(4, np.int32), tex)
    occ = counts > 0
    per = np.array([round(0.5 * 0.2 * 65536), round(0.75 * 0.4 * 65536), 65536], np.int64)
    val = np.float32(0.5) * (np.float32(51) / np.float32(255)), np.float32(0.75) * (np.float32(102) / np.float32(255))
    per[0] = int(np.rint(np.float64(val[0] * np.float32(65536))))
    per[1] = int(np.rint(np.float64(val[1] * np.float32(65536))))
    assert np.array_equal(sums[occ, :3], counts[occ, None].astype(np.int64) * per[None, :])


def test_textured_voxelize_bad_map_rejected(oracle_mod):
    n, g0, E, verts, idx, tri_mat, kd, mat_map, textures = _textured_case(1)
    with pytest.raises(ValueError):
        oracle_mod.voxelize(n, g0, E, verts, idx, tri_mat, kd, np.array([0, -1, 2, 0], np.int32), textures)


# ---------------------------------------------------------------------------
# CPU backend of include/vct.h
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def cpu_lib(oracle_mod):
    from vct import _lib
    return _lib.bind(C.CDLL(oracle_mod.CPU_BACKEND))


def test_cpu_backend_textured_state_and_errors(cpu_lib, oracle_mod):
    from vct import Context, VctError
    n, g0, E, verts, idx, tri_mat, kd, mat_map, textures = _textured_case(2)
    ctx = Context(n, g0, E, lib=cpu_lib)
    with pytest.raises(VctError, match="EINVAL"):          # no textures set yet
        ctx.voxelize(verts, idx, tri_mat, kd, material_map=mat_map)
    with pytest.raises(VctError, match="EINVAL"):
        ctx.set_textures([np.zeros((0, 4, 4), np.uint8)])
    ctx.set_textures(textures)
    with pytest.raises(VctError, match="EINVAL"):          # uv_offset past the record
        ctx.voxelize(verts, idx, tri_mat, kd, material_map=mat_map, uv_offset=52)
    with pytest.raises(VctError, match="EINVAL"):
        ctx.voxelize(verts, idx, tri_mat, kd, material_map=np.array([0, 5, 1, 0], np.int32))
    ctx.voxelize(verts, idx, tri_mat, kd, material_map=mat_map)
    sums, counts = ctx.download_accum()
    rs, rc = oracle_mod.voxelize(n, g0, E, verts, idx, tri_mat, kd, mat_map, textures)
    assert np.array_equal(sums, rs) and np.array_equal(counts, rc)
    ctx.close()


def test_cpu_backend_gbuffer_albedo_at_hit_uv(cpu_lib, oracle_mod):
    """G-buffer albedo = Kd x T(uv of the hit): recomputed here from the hit position
    (barycentrics in float64, so only to within float rounding of the UV)."""
    from vct import Context, scenes
    from vct.camera import Camera
    s = scenes.showroom(1)
    v, i, m, k = s.arrays()
    g = np.load(os.path.join(GOLD, "tex_nanosuit.npz"))
    names = [p for _, p in scenes.NANOSUIT_MATERIALS]
    tex = [g["crop_" + p] for p in names]
    g0, E = scenes.grid_for_unit_box(32)
    ctx = Context(32, g0, E, lib=cpu_lib)
    ctx.set_textures(tex)
    ctx.voxelize(v, i, m, k, material_map=s.material_map(names))
    cam = Camera()
    w, h = 48, 32
    pos, nrm, alb = (np.zeros((h, w, 4), np.float32) for _ in range(3))
    ctx.gbuffer_raycast_device(cam, w, h, 0.1, pos.ctypes.data, nrm.ctypes.data, alb.ctypes.data)
    P = v[:, :3].astype(np.float64)[i.reshape(-1, 3)]
    UV = v[:, 6:8].astype(np.float64)[i.reshape(-1, 3)]
    mm = s.material_map(names)
    checked = 0
    for y in range(h):
        for x in range(w):
            if pos[y, x, 3] == 0:
                continue
            p = pos[y, x, :3].astype(np.float64)
            # the triangles holding p (an edge or a corner between faces holds several: skipped)
            cands = []
            for t in range(P.shape[0]):
                a, b, c = P[t]
                nrm_t = np.cross(b - a, c - a)
                ln = np.linalg.norm(nrm_t)
                if ln == 0 or abs(np.dot(p - a, nrm_t / ln)) > 1e-4:
                    continue
                bb, *_ = np.linalg.lstsq(np.array([b - a, c - a]).T, p - a, rcond=None)
                if bb.min() >= -1e-3 and bb.sum() <= 1 + 1e-3:
                    cands.append(t)
            bt = cands[0] if len(cands) == 1 else -1
            if bt < 0 or mm[m[bt]] < 0:
                continue
            a, b, c = P[bt]
            bb, *_ = np.linalg.lstsq(np.array([b - a, c - a]).T, p - a, rcond=None)
            uv = UV[bt, 0] + bb[0] * (UV[bt, 1] - UV[bt, 0]) + bb[1] * (UV[bt, 2] - UV[bt, 0])
            tx = tex[mm[m[bt]]]
            expect = k[m[bt], :3] * oracle_mod.tex_sample(tx, uv[0], uv[1])
            # the texel gradient bounds the error from the float32 UV
            assert np.allclose(alb[y, x, :3], expect, atol=0.02), (x, y, alb[y, x], expect)
            checked += 1
    assert checked > 200
    ctx.close()
