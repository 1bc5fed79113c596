#!/usr/bin/env python3
"""K1-K3 timing on device-resident geometry (run under rocprofv3 --kernel-trace
--stats for the per-kernel split).

    python tools/k1_bench.py [--scene courtyard] [--n 256] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="courtyard")
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    from vct import Context, scenes
    s = scenes.SCENES[a.scene]()
    v, i, m, k = s.arrays()
    dev = torch.device("cuda")
    geo = (torch.from_numpy(v).to(dev), torch.from_numpy(i.astype(np.int32)).to(dev),
           torch.from_numpy(m.astype(np.int32)).to(dev), torch.from_numpy(k).to(dev))
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ts = {"k1": [], "k2": [], "k3": []}
    for r in range(a.reps + 1):
        for key, fn in (("k1", lambda: ctx.voxelize_device(*geo)),
                        ("k2", lambda: ctx.inject_directional(scenes.LIGHT_DIR)), ("k3", ctx.build_mips)):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            if r:
                ts[key].append((time.perf_counter() - t) * 1e3)
    import hashlib
    ao, nm = ctx.download_voxels()
    hs = hashlib.sha256(ao.tobytes() + nm.tobytes() + ctx.download_level(0).tobytes())
    if a.n <= 256:                     # the raw accumulators too (8.6 GB of records at 512^3)
        sums, counts = ctx.download_accum()
        hs.update(sums.tobytes() + counts.tobytes())
    h = hs.hexdigest()[:16]
    print(json.dumps({"scene": a.scene, "n": a.n, "tris": int(s.n_tri), "lib": os.path.basename(os.environ.get("VCT_LIB", "")),
                      **{k2: round(sorted(x)[len(x) // 2], 3) for k2, x in ts.items()}, "hash": h}))


if __name__ == "__main__":
    main()
