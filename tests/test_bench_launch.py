"""bench.py's own N-rank launch on the CPU: `--gpus N` without a torch.distributed
environment starts the N ranks itself (one child per rank, nothing touches a GPU
in the parent) and rank 0 prints ONE JSON line.  `--dry-run` swaps the HIP trace
for a pattern-writing stand-in over gloo, so the launcher, the process group, the
exchange in both modes and the max-over-ranks reduction run here; the assembled
frames are checked exactly."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n,exchange", [(2, "present"), (3, "allgather")])
def test_bench_spawns_ranks_dry_run(n, exchange):
    d = _run("--gpus", str(n), "--dry-run", "--steps", "2", "--width", "200", "--height", "130",
             "--exchange", exchange)
    assert d["n_gpus"] == n and d["dry_run"] is True and d["value"] is None
    assert d["exchange"] == exchange
    assert all(v["frame_ok"] for v in d["exchange_check"].values())
    for k in ("trace_ms_max_rank", "gather_ms", "allgather_ms", "metric", "unit", "scaling"):
        assert k in d


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=REPO)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_roofline_from_profile(tmp_path):
    """The bound is the larger of the VALU-issue and HBM fractions; a profile of
    another library build is refused (no stale counters)."""
    sys.path.insert(0, REPO)
    import bench
    key = bench.profile_key(256, 1920, 1080, "atrium", "scene", 9, True, 0, 1)
    rec = {"lib_sha256": bench.lib_sha256(), "SQ_INSTS_VALU": 6.0e8, "SQ_INSTS_SALU": 3.0e8,
           "hbm_bytes_per_launch": 7.0e8, "duration_ms": 1.3}
    p = tmp_path / "k.json"
    p.write_text(json.dumps({key: rec}))
    got, why = bench.load_profile(str(p), key)
    assert got == rec and why is None
    r = bench.roofline(got, why, 1.0, 1000, 10, str(p), key)
    assert r["bound"] == "issue (VALU)" and r["frac"] == pytest.approx(6.0e8 / 1e-3 / 1e9 / bench.VALU_PEAK_G, abs=1e-4)
    assert 0 < r["frac"] <= 1 and r["hbm"]["frac"] == pytest.approx(0.7 / 8.0, abs=1e-4)
    assert r["gather_bytes"] == 1000 * 16 + 10 * 80
    r = bench.roofline(dict(rec, SQ_INSTS_SALU=5.0e8), None, 1.0, 1000, 10, str(p), key)
    assert r["bound"] == "issue (scalar)" and r["frac"] == pytest.approx(5.0e8 / 1e-3 / 1e9 / bench.SALU_PEAK_G, abs=1e-4)
    r = bench.roofline(dict(rec, hbm_bytes_per_launch=7.9e9), None, 1.0, 1000, 10, str(p), key)
    assert r["bound"] == "hbm" and r["frac"] == pytest.approx(7.9 / 8.0, abs=1e-4)
    p.write_text(json.dumps({key: dict(rec, lib_sha256="0" * 64)}))
    got, why = bench.load_profile(str(p), key)
    assert got is None and "another library build" in why
    r = bench.roofline(got, why, 1.0, 1000, 10, str(p), key)
    assert r["frac"] is None and r["note"]


def test_k3_relight_bytes():
    """bench.k3_relight_bytes: a relight K3 build reads / writes the first launch's bytes
    only for blocks (16 x 16 x 8 level-0 voxels at the default depth) holding an occupied
    voxel; every block live = the full build's algorithmic bytes plus the later launches'
    read of level 3, none live = only the later launches (level 3 read, levels 4..L
    written)."""
    import math
    import numpy as np
    sys.path.insert(0, REPO)
    import bench
    n = 64
    L = int(math.log2(n))
    full = n ** 3 * 16 + sum(6 * (n >> l) ** 3 * 16 for l in range(1, L + 1))
    rest = 6 * (n >> 3) ** 3 * 16 + sum(6 * (n >> l) ** 3 * 16 for l in range(4, L + 1))
    occ = np.zeros((n, n, n), np.float32)
    assert bench.k3_relight_bytes(occ, n) == (rest, 0.0)
    occ[::8, ::16, ::16] = 1.0                       # one voxel in every block
    assert bench.k3_relight_bytes(occ, n) == (full + 6 * (n >> 3) ** 3 * 16, 1.0)
    occ[:] = 0.0
    occ[0, 0, 0] = occ[n - 1, n - 1, n - 1] = 1.0      # two of (n/16)^2 (n/8) blocks
    b, frac = bench.k3_relight_bytes(occ, n)
    assert frac == 2 / ((n // 16) ** 2 * (n // 8)) and rest < b < full
