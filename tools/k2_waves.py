#!/usr/bin/env python3
"""Per-wave timeline of one K2 shadow-walk launch (timeline build, `make wv`).

    make -C voxel-based-global-illumination_amd wv
    VCT_K2_WALK=160256 python tools/k2_waves.py [--scene atrium] [--n 256]

Records (start, end) of every k2_walk wave that had work (s_memrealtime, 100 MHz) and
reports the launch span, the wave-duration distribution, how many waves are in flight
over the span, and when the waves end: whether the launch is bound by its longest waves
(a tail) or by the work of all of them.
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "voxel-based-global-illumination_amd")
os.environ["VCT_LIB"] = os.path.join(PKG, "vct", "libvct_hip_wv.so")
sys.path[:0] = [REPO, PKG]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="atrium")
    ap.add_argument("--n", type=int, default=256)
    a = ap.parse_args()
    import numpy as np
    import torch
    from vct import Context, _lib, scenes
    lib = _lib.load()
    lib.vct_debug_k2_waves.restype = C.c_int
    lib.vct_debug_k2_waves.argtypes = [C.c_void_p, C.c_int]
    lib.vct_debug_k2_waves_clear.restype = C.c_int
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    for _ in range(3):
        ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    torch.cuda.synchronize()
    assert lib.vct_debug_k2_waves_clear() == 0
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    torch.cuda.synchronize()
    nw = 1 << 16
    buf = np.zeros((nw, 3), np.uint64)
    assert lib.vct_debug_k2_waves(buf.ctypes.data_as(C.c_void_p), nw) == nw
    used = np.flatnonzero(buf[:, 1])
    t = buf[used].astype(np.int64)
    t0 = t[:, 0].min()
    st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0      # microseconds
    dur = en - st
    span = float(en.max())
    ends = np.sort(en)
    ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([en, -np.ones_like(en)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    infl = np.cumsum(ev[:, 1])
    qs = [0.1, 0.25, 0.5, 0.75, 0.9]
    out = {
        "scene": a.scene, "n": a.n, "walk": os.environ.get("VCT_K2_WALK", "default"),
        "waves": int(len(used)), "span_us": round(span, 1),
        "last_start_us": round(float(st.max()), 1),
        "wave_us_mean_p50_p90_p99_max": [round(float(dur.mean()), 1)] +
                                        [round(float(np.percentile(dur, q)), 1) for q in (50, 90, 99)] +
                                        [round(float(dur.max()), 1)],
        "sum_wave_us": round(float(dur.sum()), 1),
        "mean_in_flight": round(float(dur.sum() / span), 1),
        "max_in_flight": int(infl.max()),
        "in_flight_at_span_frac": {str(q): int(infl[np.searchsorted(ev[:, 0], q * span) - 1]) for q in qs},
        "span_frac_when_waves_ended": {str(q): round(float(ends[int(q * (len(ends) - 1))] / span), 3)
                                       for q in (0.5, 0.9, 0.99)},
    }
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
