#!/usr/bin/env python3
"""Golden vectors for the scene loader: what assimp 3.3
returns for the reference's import flags on procedural OBJ/MTL files.

The reference's Model::loadModel (assets/code/scene/model.cpp:21-148) reads a
model with Assimp::Importer::ReadFile(path, aiProcess_Triangulate |
aiProcess_FlipUVs | aiProcess_CalcTangentSpace) (model.cpp:24) and copies each
aiMesh into a 56-byte Vertex array + u32 indices + Material(Ka, Kd, Ks).  The
reference's own assimp is an MSVC import library (unusable here); this image
carries assimp 3.3 statically linked into
/opt/conda/plugins/sceneparsers/libassimpsceneimport.so.  This
script calls its C API (aiImportFile, same flags) through ctypes in THIS
container and stores inputs and outputs as tests/golden/obj_<case>.npz:

  obj, mtl            the OBJ / MTL text (uint8)
  mat_names           material names joined by '\\n' (uint8)
  mat_ka/kd/ks        [n_mat, 4] float32 (r, g, b, 1) as model.cpp:48-53 builds them
  n_meshes            int
  mesh<i>_verts       [n_verts, 14] float32: Position, Normal, TexCoords, Tangent, Bitangent
  mesh<i>_idx         [n_idx] uint32 (faces in order, model.cpp:126-133)
  mesh<i>_mat         material index

tests/test_scene_loader.py compares the repo's loader (vct/libvct_host.so,
include/vct_host.h) with these files; assimp itself never ships or runs on
the GPU box.

    python tests/golden/make_obj_golden.py
"""
import ctypes as C
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ASSIMP = "/opt/conda/plugins/sceneparsers/libassimpsceneimport.so"
FLAGS = 0x1 | 0x8 | 0x800000     # aiProcess_CalcTangentSpace | aiProcess_Triangulate | aiProcess_FlipUVs


class V3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Face(C.Structure):
    _fields_ = [("n", C.c_uint), ("idx", C.POINTER(C.c_uint))]


class AiString(C.Structure):      # assimp 3.3: size_t length
    _fields_ = [("length", C.c_size_t), ("data", C.c_char * 1024)]


class Mesh(C.Structure):          # assimp 3.3 aiMesh prefix (include/assimp/mesh.h)
    _fields_ = [("prim", C.c_uint), ("nv", C.c_uint), ("nf", C.c_uint), ("v", C.POINTER(V3)),
                ("n", C.POINTER(V3)), ("t", C.POINTER(V3)), ("b", C.POINTER(V3)), ("col", C.c_void_p * 8),
                ("uv", C.POINTER(V3) * 8), ("nuv", C.c_uint * 8), ("faces", C.POINTER(Face)),
                ("nbones", C.c_uint), ("bones", C.c_void_p), ("mat", C.c_uint)]


class Scene(C.Structure):
    _fields_ = [("flags", C.c_uint), ("root", C.c_void_p), ("nm", C.c_uint), ("meshes", C.POINTER(C.POINTER(Mesh))),
                ("nmat", C.c_uint), ("mats", C.POINTER(C.c_void_p))]


class Col4(C.Structure):
    _fields_ = [("r", C.c_float), ("g", C.c_float), ("b", C.c_float), ("a", C.c_float)]


# ---------------------------------------------------------------------------
# procedural inputs
# ---------------------------------------------------------------------------
MTL = """newmtl red
Ka 0.1 0.0 0.0
Kd 0.63 0.065 0.05
Ks 0.0 0.0 0.0
newmtl white
Kd 0.725 0.71 0.68
newmtl green
Kd 0.14 0.45 0.091
Ks 0.2 0.2 0.2
"""

CUBE = """mtllib scene.mtl
o box
v -1 -1 -1
v 1 -1 -1
v 1 1 -1
v -1 1 -1
v -1 -1 1
v 1 -1 1
v 1 1 1
v -1 1 1
vt 0 0
vt 1 0
vt 1 1
vt 0 1
vn 0 0 -1
vn 0 0 1
vn 1 0 0
vn -1 0 0
vn 0 1 0
vn 0 -1 0
usemtl red
f 1/1/1 4/4/1 3/3/1 2/2/1
f 5/1/2 6/2/2 7/3/2 8/4/2
usemtl white
f 2/1/3 3/2/3 7/3/3 6/4/3
f 1/1/4 5/2/4 8/3/4 4/4/4
usemtl green
f 4/1/5 8/2/5 7/3/5 3/4/5
f 1/1/6 2/2/6 6/3/6 5/4/6
"""

POLY = """mtllib scene.mtl
v 0 0 0
v 2 0 0
v 3 1 0
v 1.5 2.5 0
v -0.5 1.2 0
v 0 0 1
v 1 0 1
v 1 1 1
v 0 1 1
v 0.5 0.2 1
vt 0 0
vt 1 0
vt 1 1
vt 0.5 1.5
vt -0.2 0.6
vn 0 0 1
g first
usemtl white
f 1/1/1 2/2/1 3/3/1 4/4/1 5/5/1
g second
f -5/1/-1 -4/2/-1 -3/3/-1 -2/4/-1
f 6/1/1 7/2/1 10/5/1 8/3/1
usemtl red
f 6/1/1 7/2/1 8/3/1
usemtl red
f 6/1/1 8/3/1 9/4/1
usemtl white
f 6/1/1 8/3/1 9/4/1
o other
usemtl red
f 1/1/1 2/2/1 3/3/1
f 5/5/1 4/4/1 3/3/1 2/2/1 1/1/1
"""

EDGE = """v 0 0 0
v 1 0 0
v 1 1 0
v 0.3 0.3 0
vt 0 0
vt 1 0
vt 1 1
vt 0.2 0.5
vn 0 0 1
vn 0 0.1 0.995
f 1/1/1 2/2/1 3/3/1
f 1/1/2 3/3/2 4/4/1
f 1/1/1 2/2/1 3/3/1 4/4/2
usemtl nosuch
f 2/2/1 3/3/1 4/4/1
o A
f 1/1/1 2/2/1 3/3/1
o B
f 1/1/1 2/2/1 4/4/1
o A
f 2/2/1 3/3/1 4/4/1
"""

DEGEN = """v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0.6 0.4 0
v 2 0 0
vt 0.5 0.5
vt 0 0
vt 1 1
vt 2 2
vn 0 0 1
g one
f 1/1/1 2/1/1 3/1/1
f 1/2/1 2/3/1 3/4/1
f 1/2/1 2/1/1 5/3/1 4/4/1
g one
f 1/2/1 2/3/1 6/1/1 3/4/1 4/2/1 5/1/1
g two
f 1/2/1 2/1/1 3/3/1 4/4/1 2/2/1
"""


def sphere_obj(nu=16, nv=10):
    """UV sphere: quads with per-corner normals = positions (smooth), shared
    positions across faces (tangent smoothing), triangle fans at the poles,
    one concave quad, two materials."""
    lines = ["mtllib scene.mtl"]
    P, T, N = [], [], []
    for j in range(nv + 1):
        th = math.pi * j / nv
        for i in range(nu + 1):
            ph = 2 * math.pi * i / nu
            p = (math.sin(th) * math.cos(ph), math.cos(th), math.sin(th) * math.sin(ph))
            P.append(p)
            N.append(p)
            T.append((i / nu, j / nv))
    for p in P:
        lines.append("v %.6f %.6f %.6f" % p)
    for t in T:
        lines.append("vt %.6f %.6f" % t)
    for n in N:
        lines.append("vn %.6f %.6f %.6f" % n)
    k = lambda i, j: j * (nu + 1) + i + 1
    lines.append("g sphere")
    for j in range(nv):
        lines.append("usemtl %s" % ("white" if j < nv // 2 else "green"))
        for i in range(nu):
            a, b, c, d = k(i, j), k(i + 1, j), k(i + 1, j + 1), k(i, j + 1)
            if j == 0:
                lines.append("f %d/%d/%d %d/%d/%d %d/%d/%d" % (a, a, a, c, c, c, d, d, d))
            elif j == nv - 1:
                lines.append("f %d/%d/%d %d/%d/%d %d/%d/%d" % (a, a, a, b, b, b, c, c, c))
            else:
                lines.append("f %d/%d/%d %d/%d/%d %d/%d/%d %d/%d/%d" % (a, a, a, b, b, b, c, c, c, d, d, d))
    # a concave quad (dart) with its own normal
    base = len(P)
    lines += ["v 3 0 0", "v 4 1 0", "v 3 0.3 0", "v 2 1 0", "vn 0 0 1", "vt 0 0", "vt 1 1", "vt 0.5 0.3", "vt 0 1"]
    nn, tt = len(N) + 1, len(T)
    lines.append("g dart")
    lines.append("f %d/%d/%d %d/%d/%d %d/%d/%d %d/%d/%d" % (base + 1, tt + 1, nn, base + 2, tt + 2, nn,
                                                             base + 3, tt + 3, nn, base + 4, tt + 4, nn))
    return "\n".join(lines) + "\n"


def random_obj(seed=11, nverts=60, nfaces=220):
    """Random mesh: shared positions, jittered per-corner normals, random UVs,
    triangles / quads / pentagons, usemtl switches, g and o statements."""
    rng = np.random.default_rng(seed)
    lines = ["mtllib scene.mtl"]
    P = rng.uniform(-1, 1, (nverts, 3))
    for p in P:
        lines.append("v %.5f %.5f %.5f" % tuple(p))
    for t in rng.uniform(-0.5, 1.5, (nverts, 2)):
        lines.append("vt %.5f %.5f" % tuple(t))
    Nn = rng.normal(size=(nverts, 3))
    Nn /= np.linalg.norm(Nn, axis=1, keepdims=True)
    for n in Nn:
        lines.append("vn %.5f %.5f %.5f" % tuple(n))
    mats = ["red", "white", "green", "nosuch"]
    for f in range(nfaces):
        r = rng.random()
        if r < 0.05:
            lines.append("usemtl %s" % mats[rng.integers(0, 4)])
        elif r < 0.07:
            lines.append("g grp%d" % rng.integers(0, 3))
        elif r < 0.08:
            lines.append("o obj%d" % rng.integers(0, 3))
        k = 3 if rng.random() < 0.6 else 4
        # planar convex polygon: a quad on a random plane around a centre keeps quads valid
        if k == 4:
            c = rng.uniform(-1, 1, 3)
            e1 = rng.normal(size=3)
            e1 /= np.linalg.norm(e1)
            e2 = np.cross(e1, rng.normal(size=3))
            e2 /= np.linalg.norm(e2)
            quad = [c + 0.3 * (math.cos(a) * e1 + math.sin(a) * e2) for a in (0.1, 1.7, 3.3, 4.6)]
            ids = []
            for q in quad:
                lines.append("v %.5f %.5f %.5f" % tuple(q))
                nverts += 1
                ids.append(nverts)
            ti = rng.integers(1, 61, 4)
            ni = rng.integers(1, 61, 4)
            lines.append("f " + " ".join("%d/%d/%d" % (a, b, c) for a, b, c in zip(ids, ti, ni)))
        else:
            vi = rng.choice(60, 3, replace=False) + 1
            ti = rng.integers(1, 61, 3)
            ni = rng.integers(1, 61, 3)
            lines.append("f " + " ".join("%d/%d/%d" % (a, b, c) for a, b, c in zip(vi, ti, ni)))
    return "\n".join(lines) + "\n"


# diffuse maps (map_Kd) with texture options and spaces in names: the material's
# texture path as assimp reports it (aiGetMaterialTexture, aiTextureType_DIFFUSE --
# what Model::loadMaterialTextures reads, model.cpp:150-158)
MAPS_MTL = """newmtl plain
Kd 0.5 0.5 0.5
map_Kd plain.png
newmtl clamped
Kd 0.25 0.5 1
map_Kd -clamp on clamped.png
newmtl offset
Kd 1 1 1
map_Kd -o 0.5 0.25 offset.png
newmtl spaced
Kd 0.1 0.2 0.3
map_Kd sub dir/with space.png
newmtl twice
Kd 0.3 0.3 0.3
map_Kd first.png
map_Kd second.png
newmtl bumponly
Kd 0.7 0.7 0.7
map_Bump bump.png
"""
MAPS_OBJ = """mtllib scene.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
vt 0 0
vt 2 0
vt 2 -1
vt 0 3
vn 0 0 1
usemtl plain
f 1/1/1 2/2/1 3/3/1
usemtl clamped
f 1/1/1 3/3/1 4/4/1
usemtl offset
f 2/2/1 3/3/1 4/4/1
usemtl spaced
f 1/1/1 2/2/1 4/4/1
usemtl twice
f 1/4/1 2/3/1 3/2/1
usemtl bumponly
f 4/1/1 3/2/1 2/3/1
"""

CASES = {"cube": CUBE, "poly": POLY, "edge": EDGE, "degen": DEGEN, "sphere": sphere_obj(),
         "random": random_obj()}

# The reference's own material library (assets/model/test/nanosuit.mtl, Blender
# export: Ns/Ni/d/illum/map_* lines) is data: it is stored in the fixture as the
# MTL input of one case, with a procedural mesh that uses its materials by name.
REF_MTL = "/root/reference/assets/model/test/nanosuit.mtl"
NANO_OBJ = """mtllib scene.mtl
o Visor
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0.5 0.5 1
vt 0 0
vt 1 0
vt 1 1
vt 0 1
vn 0 0 -1
vn 0 0.7071 0.7071
usemtl Glass
f 1/1/1 2/2/1 3/3/1 4/4/1
usemtl Helmet
f 1/1/2 2/2/2 5/3/2
f 2/2/2 3/3/2 5/4/2
o Body
usemtl Body
f 3/1/2 4/2/2 5/3/2
usemtl Arm
f 4/1/2 1/2/2 5/3/2
usemtl Leg
f 1/1/1 3/3/1 2/2/1
"""


def import_with_assimp(lib, path):
    sc = lib.aiImportFile(path.encode(), FLAGS)
    if not sc:
        raise RuntimeError(lib.aiGetErrorString())
    s = sc.contents
    out = {"n_meshes": np.int64(s.nm)}
    names, ka, kd, ks, dif = [], [], [], [], []
    for i in range(s.nmat):
        m = s.mats[i]
        st = AiString()
        lib.aiGetMaterialString(m, b"?mat.name", 0, 0, C.byref(st))
        names.append(st.data[:st.length].decode())
        for key, dst in ((b"$clr.ambient", ka), (b"$clr.diffuse", kd), (b"$clr.specular", ks)):
            c = Col4(0, 0, 0, 0)
            lib.aiGetMaterialColor(m, key, 0, 0, C.byref(c))
            dst.append((c.r, c.g, c.b, 1.0))   # model.cpp:48-53: vec4(color.rgb, 1.0)
        # loadMaterialTextures(aMat, aiTextureType_DIFFUSE, ..) (model.cpp:57, :153-158)
        path = ""
        if lib.aiGetMaterialTextureCount(m, 1) > 0:
            st = AiString()
            lib.aiGetMaterialTexture(m, 1, 0, C.byref(st), None, None, None, None, None, None)
            path = st.data[:st.length].decode()
        dif.append(path)
    out["mat_names"] = np.frombuffer("\n".join(names).encode(), np.uint8)
    out["mat_diffuse"] = np.frombuffer("\n".join(dif).encode(), np.uint8)
    out["mat_ka"], out["mat_kd"], out["mat_ks"] = (np.array(x, np.float32) for x in (ka, kd, ks))
    for i in range(s.nm):
        m = s.meshes[i].contents
        nv = m.nv
        arr = np.zeros((nv, 14), np.float32)
        for j in range(nv):
            arr[j, 0:3] = (m.v[j].x, m.v[j].y, m.v[j].z)
            arr[j, 3:6] = (m.n[j].x, m.n[j].y, m.n[j].z)
            if m.uv[0]:
                arr[j, 6:8] = (m.uv[0][j].x, m.uv[0][j].y)
            arr[j, 8:11] = (m.t[j].x, m.t[j].y, m.t[j].z)
            arr[j, 11:14] = (m.b[j].x, m.b[j].y, m.b[j].z)
        idx = [m.faces[f].idx[k] for f in range(m.nf) for k in range(m.faces[f].n)]
        out["mesh%d_verts" % i] = arr
        out["mesh%d_idx" % i] = np.array(idx, np.uint32)
        out["mesh%d_mat" % i] = np.int64(m.mat)
    lib.aiReleaseImport(sc)
    return out


def main():
    import tempfile
    lib = C.CDLL(ASSIMP)
    lib.aiImportFile.restype = C.POINTER(Scene)
    lib.aiImportFile.argtypes = [C.c_char_p, C.c_uint]
    lib.aiReleaseImport.argtypes = [C.POINTER(Scene)]
    lib.aiGetMaterialColor.argtypes = [C.c_void_p, C.c_char_p, C.c_uint, C.c_uint, C.POINTER(Col4)]
    lib.aiGetMaterialString.argtypes = [C.c_void_p, C.c_char_p, C.c_uint, C.c_uint, C.POINTER(AiString)]
    lib.aiGetErrorString.restype = C.c_char_p
    lib.aiGetMaterialTextureCount.argtypes = [C.c_void_p, C.c_int]
    lib.aiGetMaterialTextureCount.restype = C.c_uint
    lib.aiGetMaterialTexture.argtypes = [C.c_void_p, C.c_int, C.c_uint, C.POINTER(AiString)] + [C.c_void_p] * 6
    with tempfile.TemporaryDirectory() as d:
        cases = [(n, t, MTL) for n, t in CASES.items()] + [("maps", MAPS_OBJ, MAPS_MTL)]
        if os.path.exists(REF_MTL):
            cases.append(("nanosuit", NANO_OBJ, open(REF_MTL).read()))
        for name, text, mtl in cases:
            with open(os.path.join(d, "scene.mtl"), "w") as f:
                f.write(mtl)
            p = os.path.join(d, name + ".obj")
            with open(p, "w") as f:
                f.write(text)
            out = import_with_assimp(lib, p)
            out["obj"] = np.frombuffer(text.encode(), np.uint8)
            out["mtl"] = np.frombuffer(mtl.encode(), np.uint8)
            np.savez_compressed(os.path.join(HERE, "obj_%s.npz" % name), **out)
            print(name, "meshes", int(out["n_meshes"]),
                  "verts", sum(out["mesh%d_verts" % i].shape[0] for i in range(int(out["n_meshes"]))))


if __name__ == "__main__":
    main()
