#!/usr/bin/env python3
"""Write profiles/traffic_k4.json (HBM bytes per K4 launch) from a tools/profile.sh run.

traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per dispatch: rocprofv3
reports KiB, and on gfx950 FETCH_SIZE counts half the bytes of wide reads
(MI355X_MICROARCH.md, HBM section), so it is doubled.  bench.py attaches the
value to its roofline object when the recorded config matches the run.
usage: make_traffic_json.py <prof_dir> <n> <w> <h> <scene> <gbuffer> <variant> [out]
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d = sys.argv[1]
    n, w, h = (int(x) for x in sys.argv[2:5])
    scene, gbuf, variant = sys.argv[5], sys.argv[6], int(sys.argv[7])
    out = sys.argv[8] if len(sys.argv) > 8 else os.path.join(REPO, "profiles", "traffic_k4.json")
    s = json.loads(subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), d, os.environ.get("KSEL", "k4_trace")],
                                  capture_output=True, text=True, check=True).stdout)
    rec = {
        "config": [n, w, h, scene, gbuf, variant, 1],
        "source": os.path.relpath(d, REPO),
        "FETCH_SIZE_KiB": s.get("FETCH_SIZE"), "WRITE_SIZE_KiB": s.get("WRITE_SIZE"),
        "hbm_bytes_per_launch": int(2 * s["FETCH_SIZE"] * 1024 + s["WRITE_SIZE"] * 1024),
        "l2_hit_rate": s.get("l2_hit_rate"),
        "duration_ns_mean": s.get("duration_ns_mean"),
        "correction": "hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halves wide reads)",
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
