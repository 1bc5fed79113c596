#!/usr/bin/env python3
"""Path statistics of the LDS K4 variants (debug-counter build).

    make -C voxel-based-global-illumination_amd dbg
    python tools/dbg_counters.py [--gbuffer scene|rand] [--n 256]

Counters: 0/1 = level-A brick / gather per wave-step, 4.. = gathers per level;
16.. = per-wave phase clocks (s_memtime) of the default variant.
"""
import argparse
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "voxel-based-global-illumination_amd")
os.environ["VCT_LIB"] = os.environ.get("VCT_DBG_LIB") or os.path.join(
    PKG, "vct", "libvct_hip_clk.so" if "--clk" in sys.argv else "libvct_hip_dbg.so")
sys.path[:0] = [REPO, PKG]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--gbuffer", default="scene")
    ap.add_argument("--scene", default="atrium")
    ap.add_argument("--clk", action="store_true", help="phase clocks (make clk) instead of path counters")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--nd", type=int, default=9, help="diffuse cones (0 = the specular cone alone)")
    ap.add_argument("--spec", type=int, default=1, help="specular cone on/off")
    a = ap.parse_args()
    import torch
    from vct import Context, _lib, scenes
    from vct.camera import Camera
    lib = _lib.load()
    lib.vct_debug_counters.restype = C.c_int
    lib.vct_debug_counters.argtypes = [C.c_void_p, C.c_int]
    ctr = (C.c_ulonglong * 56)()
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E, n_diffuse=a.nd, specular=bool(a.spec))
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    s = scenes.SCENES[a.scene]()
    ctx.voxelize(*s.arrays())
    ctx.inject_directional(scenes.LIGHT_DIR)
    ctx.build_mips()
    dev = torch.device("cuda")
    cam = Camera()
    if a.gbuffer == "scene":
        gb = [torch.empty((a.h, a.w, 4), device=dev) for _ in range(3)]
        ctx.gbuffer_raster_device(cam, a.w, a.h, scenes.ROUGHNESS, *gb)
    else:
        ao, nm = ctx.download_voxels()
        gb = [torch.from_numpy(x).to(dev) for x in scenes.gbuffer_rand(ao, nm, g0, E, a.w, a.h)]
    d = torch.empty((a.h, a.w, 4), device=dev)
    sp = torch.empty((a.h, a.w, 4), device=dev)
    for v in [int(x, 0) for x in a.variants.split(",")]:
        ctx.trace_device(*gb, a.w, a.h, cam.position, d, sp, variant=v)   # warm caches, step tables
        torch.cuda.synchronize()
        lib.vct_debug_counters(ctr, 1)
        ctx.trace_device(*gb, a.w, a.h, cam.position, d, sp, variant=v)
        torch.cuda.synchronize()
        lib.vct_debug_counters(ctr, 1)
        c = list(ctr)
        print(f"variant {v}: level-A brick {c[0]} / gather {c[1]} / staged {c[2]} / cache hit {c[3]}; "
              f"gathers per level: {c[4:15]}")
        print(f"  level-A brick samples: zero brick {c[17]} / nonzero {c[15]}")
        if not a.clk:
            print(f"  level B: hit {c[26]} / staged {c[27]} / gather {c[28]} / not sampled {c[31]}; "
                  f"faces-mode brick samples A {c[29]} / B {c[30]}")
            print(f"  empty-space maps: level-A misses skipped {c[40]}")
            print(f"  level-B stagings: combined-face march {c[41]} / faces {c[42]} / iso {c[50]}; "
                  f"while level A hit the cache {c[43]}")
            print(f"  iso / combined-face gathers {c[53]}: would fit 5^3 {c[51]} / 6^3 {c[52]} / 8x8x3 {c[54]} / "
                  f"a box of <= 216 texels {c[55]}")
        print(f"  wave-steps: table {c[44]} / per-lane {c[46]}; active lanes {c[45]} "
              f"({c[45] / max(c[44] + c[46], 1):.1f} per wave-step), valid-pixel lanes {c[47] / max(c[44] + c[46], 1):.1f}")
        print(f"  gather reasons: faces not uniform {c[16]}; footprint span (level 0) <=3/<=5/<=9/more {c[18:22]}"
              f"; (level>0) {c[22:26]}")
        if a.clk:
            print(f"  longest wave {c[39]} cycles; wave durations (2^k cycles: count):",
                  ", ".join(f"{10 + k}:{c[k]}" for k in range(22) if c[k]))
            lt = max(c[30], 1)
            nmid = sum(c[8:10])
            print(f"  waves >= 2^20 cycles: {c[22]}, {c[23] / max(c[22], 1):.0f} steps each; "
                  f"waves 2^18..2^20: {nmid}, {c[31] / max(nmid, 1):.0f} steps each")
            print("  waves >= 2^20 cycles, phase split:",
                  ", ".join(f"{n} {100.0 * c[24 + i] / lt:.1f}%" for i, n in
                            enumerate(["head", "geometry", "staging", "lds-sample", "fallback", "tail"])))
        names = ["head", "geometry", "staging", "lds-sample", "fallback", "tail", "kernel"]
        tot = max(c[32 + 6], 1)
        print("  phase cycles (sum over waves):",
              ", ".join(f"{n} {c[32 + i] / 1e9:.3f}G ({100.0 * c[32 + i] / tot:.1f}%)" for i, n in enumerate(names)))


if __name__ == "__main__":
    main()
