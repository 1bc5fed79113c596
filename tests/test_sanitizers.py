"""AddressSanitizer + UBSan on the host-side C/C++.

tests/native/Makefile builds two executables with -fsanitize=address,undefined
-fno-sanitize-recover=all (any overflow, use-after-free, leak or UB aborts):
* obj_fuzz_driver: the OBJ/MTL loader (host/scene.cpp, which parses untrusted
  files), the placement helpers and the camera, fed hypothesis-generated
  OBJ/MTL files: degenerate and huge polygons, negative / out-of-range / zero
  indices, partial `v/vt/vn` triples, missing or broken .mtl files, undefined
  materials, non-finite and out-of-range numbers, junk lines;
* cpu_backend_driver: one include/vct.h call sequence on the CPU oracle backend
  (oracle/vct_cpu_backend.c + vct_oracle.c, OpenMP on): voxelize / inject / mips /
  trace / tiled + packed untile / composite / downloads and the error paths.
"""
import os
import subprocess

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "oracle", "_build", "san")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
           OMP_NUM_THREADS="4")


@pytest.fixture(scope="module")
def drivers():
    subprocess.run(["make", "-C", os.path.join(REPO, "tests", "native")], check=True, capture_output=True)
    return os.path.join(SAN, "obj_fuzz_driver"), os.path.join(SAN, "cpu_backend_driver")


def _run(cmd):
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=ENV)
    bad = [m for m in ("AddressSanitizer", "runtime error", "LeakSanitizer") if m in p.stderr]
    assert p.returncode == 0 and not bad, (p.returncode, bad, p.stderr[-3000:])
    return p.stdout


@pytest.mark.parametrize("n", [4, 16, 32])
def test_cpu_backend_under_sanitizers(drivers, n):
    assert _run([drivers[1], str(n)]).startswith("ok")


NUM = st.one_of(st.floats(allow_nan=True, allow_infinity=True, width=32).map(repr),
                st.integers(-10 ** 12, 10 ** 12).map(str),
                st.sampled_from(["1e400", "-1e-400", "nan", "-inf", "0x1p3", "", "--1", "1.2.3", "+.5", "7e", "1e+"]))
IDX = st.one_of(st.integers(-40, 40).map(str), st.sampled_from(["", "0", "99999999999", "-99999999999", "x"]))
VREF = st.one_of(IDX, st.tuples(IDX, IDX).map("/".join), st.tuples(IDX, IDX, IDX).map("/".join),
                 st.tuples(IDX, IDX).map(lambda t: f"{t[0]}//{t[1]}"))
LINE = st.one_of(
    st.lists(NUM, min_size=0, max_size=5).map(lambda xs: "v " + " ".join(xs)),
    st.lists(NUM, min_size=0, max_size=3).map(lambda xs: "vt " + " ".join(xs)),
    st.lists(NUM, min_size=0, max_size=4).map(lambda xs: "vn " + " ".join(xs)),
    st.lists(VREF, min_size=0, max_size=14).map(lambda xs: "f " + " ".join(xs)),
    st.integers(3, 300).map(lambda k: "f " + " ".join(str(i % 9 + 1) for i in range(k))),   # huge polygons
    st.sampled_from(["usemtl red", "usemtl undefined", "usemtl", "o obj", "g grp a b", "s 1", "s off",
                     "mtllib scene.mtl", "mtllib missing.mtl", "mtllib", "# comment", "", "\\", "v 1 2 3 \\",
                     "l 1 2 3", "p 1", "vp 0.5", "\t v 1 2 3", "f 1 2 3 # tail"]),
    st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=40),
)
MTL = st.lists(st.one_of(
    st.sampled_from(["newmtl red", "newmtl", "newmtl other", "Ka", "illum 2", "map_Kd tex.png", "d 0.5", ""]),
    st.tuples(st.sampled_from(["Kd", "Ka", "Ks", "Ke"]), st.lists(NUM, max_size=4)).map(lambda t: t[0] + " " + " ".join(t[1])),
    st.text(max_size=30)), max_size=12)


@settings(max_examples=int(os.environ.get("VCT_FUZZ_EXAMPLES", "80")), deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture,
                                                                   HealthCheck.too_slow])
@given(obj=st.lists(LINE, min_size=0, max_size=60), mtl=st.one_of(st.none(), MTL),
       base=st.lists(st.tuples(NUM, NUM, NUM), min_size=0, max_size=8))
def test_obj_loader_fuzz_under_sanitizers(drivers, tmp_path_factory, obj, mtl, base):
    d = tmp_path_factory.mktemp("fz")
    lines = ["mtllib scene.mtl"] + [f"v {x} {y} {z}" for x, y, z in base] + obj
    (d / "scene.obj").write_text("\n".join(lines) + "\n", errors="surrogatepass")
    if mtl is not None:
        (d / "scene.mtl").write_text("\n".join(mtl) + "\n", errors="surrogatepass")
    (d / "empty.obj").write_text("")
    (d / "nomtl.obj").write_text("mtllib nothere.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\nusemtl ghost\nf 3 2 1\n")
    out = _run([drivers[0], str(d / "scene.obj"), str(d / "empty.obj"), str(d / "nomtl.obj"), str(d / "absent.obj")])
    assert out.startswith("loaded")


_PNG_CASES = None


def _png_cases():
    global _PNG_CASES
    if _PNG_CASES is None:
        import numpy as np
        g = np.load(os.path.join(REPO, "tests", "golden", "tex_png_cases.npz"))
        _PNG_CASES = [g["png_" + n].tobytes() for n in g["names"]]
    return _PNG_CASES


@settings(max_examples=int(os.environ.get("VCT_FUZZ_EXAMPLES", "80")), deadline=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(case=st.integers(0, 116), edits=st.lists(st.tuples(st.integers(0, 10 ** 6), st.integers(0, 255)), max_size=8),
       cut=st.one_of(st.none(), st.integers(0, 10 ** 6)))
def test_png_decoder_fuzz_under_sanitizers(drivers, tmp_path_factory, case, edits, cut):
    """host/png.cpp (untrusted texture files) on corrupted PNGs: byte edits anywhere
    (chunk lengths, IHDR fields, filter bytes, compressed data) and truncations."""
    blob = bytearray(_png_cases()[case % len(_png_cases())])
    for at, val in edits:
        blob[at % len(blob)] = val
    if cut is not None:
        blob = blob[:cut % (len(blob) + 1)]
    d = tmp_path_factory.mktemp("png")
    (d / "x.png").write_bytes(bytes(blob))
    (d / "y.png").write_bytes(_png_cases()[(case + 1) % len(_png_cases())])
    assert _run([drivers[0], "--png", str(d / "x.png"), str(d / "y.png")]).startswith("decoded")


def test_obj_loader_sanitized_on_golden_files(drivers):
    """Every OBJ the loader parity tests use, under the sanitizers."""
    import glob
    import tempfile
    import numpy as np
    with tempfile.TemporaryDirectory() as tmp:
        files = []
        for f in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "obj_*.npz"))):
            z = np.load(f, allow_pickle=False)
            sub = os.path.join(tmp, os.path.basename(f)[:-4])
            os.makedirs(sub)
            with open(os.path.join(sub, "scene.obj"), "wb") as fh:
                fh.write(z["obj"].tobytes())
            if "mtl" in z.files:
                with open(os.path.join(sub, "scene.mtl"), "wb") as fh:
                    fh.write(z["mtl"].tobytes())
            files.append(os.path.join(sub, "scene.obj"))
        out = _run([drivers[0]] + files)
        assert out.startswith(f"loaded {len(files)} ")
