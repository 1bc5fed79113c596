#!/usr/bin/env python3
"""Per-wave timeline of one K4 launch (clock build) and schedule replays.

    make -C voxel-based-global-illumination_amd clk
    python tools/wave_sched.py [--scene atrium] [--variant 0]

Records (start, end) of every wave (s_memrealtime, 100 MHz) of one launch and
reports: the launch span, the sum of wave durations, slot occupancy, and what a
greedy list schedule over S concurrent wave slots would give for the
dispatch (blockIdx) order and for longest-first (LPT) order of the same
durations (an upper bound on what reordering the blocks could buy).
"""
import argparse
import ctypes as C
import heapq
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "voxel-based-global-illumination_amd")
os.environ["VCT_LIB"] = os.path.join(PKG, "vct", "libvct_hip_wv.so" if "--wv" in sys.argv else "libvct_hip_clk.so")
sys.path[:0] = [REPO, PKG]


def list_schedule(durs, slots):
    h = [0.0] * slots
    heapq.heapify(h)
    end = 0.0
    for d in durs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + d)
        end = max(end, t + d)
    return end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="atrium")
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--variant", type=lambda x: int(x, 0), default=0)
    ap.add_argument("--slots", type=int, default=256 * 16)
    ap.add_argument("--wv", action="store_true", help="timeline-only build (make wv), no phase clocks")
    ap.add_argument("--world", type=int, default=1, help="trace rank --rank's tiles of a --world split")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--parts", type=int, default=0, help="cone parts of the launch (per-part wave stats)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from vct import Context, _lib, scenes
    from vct.camera import Camera
    lib = _lib.load()
    lib.vct_debug_waves.restype = C.c_int
    lib.vct_debug_waves.argtypes = [C.c_void_p, C.c_int]
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR)
    ctx.build_mips()
    dev = torch.device("cuda")
    cam = Camera()
    gb = [torch.empty((a.h, a.w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, a.w, a.h, scenes.ROUGHNESS, *gb)
    from vct.multi import tiles_for_rank
    opx = tiles_for_rank(a.w, a.h, a.rank, a.world) * 4096 if a.world > 1 else a.w * a.h
    d = torch.empty((opx, 4), device=dev)
    sp = torch.empty((opx, 4), device=dev)
    if a.world == 1 and not a.variant & (0x8000 | 0x4000000):
        # a one-rank frame's tuner alternates screen order and ray reordering while it times
        # them: their grids differ, so one launch's records would be mixed with the other's
        a.variant |= 0x4000000
    for _ in range(64 if a.world > 1 else 2):   # settle the form of this launch, then record the last
        ctx.trace_device(*gb, a.w, a.h, cam.position, d, sp, variant=a.variant, tile_rank=a.rank,
                         tile_world=a.world, tile_compact=a.world > 1)
        torch.cuda.synchronize()
    nw = 1 << 18
    buf = np.zeros((nw, 3), np.uint64)
    lib.vct_debug_waves(buf.ctypes.data_as(C.c_void_p), nw)
    used = np.flatnonzero(buf[:, 1])
    t = buf[used].astype(np.int64)
    t0 = t[:, 0].min()
    st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0      # microseconds
    dur = en - st
    span = en.max()
    half = len(used) // 2
    out = {
        "waves": int(len(used)), "span_us": round(float(span), 1),
        "sum_wave_us": round(float(dur.sum()), 1),
        "occupancy_vs_slots": round(float(dur.sum() / (span * a.slots)), 3),
        "longest_wave_us": round(float(dur.max()), 1),
        "wave_us_p50_p90_p99": [round(float(np.percentile(dur, q)), 1) for q in (50, 90, 99)],
        "first_half_mean_us": round(float(dur[used < used[half]].mean()), 1) if half else 0.0,
        "second_half_mean_us": round(float(dur[used >= used[half]].mean()), 1) if half else 0.0,
        "last_start_us": round(float(st.max()), 1),
        "replay_dispatch_order_us": round(list_schedule(dur[np.argsort(used)], a.slots), 1),
        "replay_longest_first_us": round(list_schedule(np.sort(dur)[::-1], a.slots), 1),
        "lower_bound_us": round(float(max(dur.sum() / a.slots, dur.max())), 1),
    }
    # waves in flight over time, and per-CU concurrency
    ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([en, -np.ones_like(en)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    infl = np.cumsum(ev[:, 1])
    hw = buf[used, 2].astype(np.uint64)
    hwid = (hw & 0xffffffff).astype(np.int64)
    xcc = (hw >> 32).astype(np.int64) & 0xf
    cu = (hwid >> 8) & 0xf
    se = (hwid >> 13) & 0x7
    key = xcc * 1000 + se * 100 + cu
    ucu = np.unique(key)
    out["distinct_cus"] = int(len(ucu))
    out["max_in_flight"] = int(infl.max())
    qs = [0.1, 0.25, 0.5, 0.75, 0.9]
    out["in_flight_at_span_frac"] = {str(q): int(infl[np.searchsorted(ev[:, 0], q * span) - 1]) for q in qs}
    # max concurrent waves on one CU
    mx = 0
    for k in ucu[:64]:
        m = key == k
        e2 = np.concatenate([np.stack([st[m], np.ones(m.sum())], 1), np.stack([en[m], -np.ones(m.sum())], 1)])
        e2 = e2[np.lexsort((e2[:, 1], e2[:, 0]))]
        mx = max(mx, int(np.cumsum(e2[:, 1]).max()))
    out["max_waves_on_one_cu(first 64 CUs)"] = mx
    out["waves_per_xcc"] = np.bincount(xcc, minlength=8).tolist()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    out["xcd_last_end_us"] = [round(float(en[xcc == x].max()), 1) if (xcc == x).any() else 0.0 for x in range(8)]
    out["xcd_sum_wave_ms"] = [round(float(dur[xcc == x].sum()) / 1e3, 1) for x in range(8)]
    if a.parts > 1:   # the launch's cone parts (dispatched one after another in blockIdx order)
        nb = (int(used.max()) + 1) // a.parts
        part = used // max(nb, 1)
        out["parts"] = [{"waves": int((part == p).sum()), "mean_us": round(float(dur[part == p].mean()), 1),
                         "p90_us": round(float(np.percentile(dur[part == p], 90)), 1),
                         "max_us": round(float(dur[part == p].max()), 1),
                         "first_start_us": round(float(st[part == p].min()), 1),
                         "last_end_us": round(float(en[part == p].max()), 1)}
                        for p in range(a.parts) if (part == p).any()]
    np.save(os.path.join(REPO, "gpurun_out", f"waves_{a.scene}_{a.variant:#x}{'_wv' if a.wv else ''}.npy"),
            buf[:int(used.max()) + 1])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
