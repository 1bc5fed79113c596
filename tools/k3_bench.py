"""K3 (mip build) timing on one GPU: the atrium at n^3, build_mips `reps` times; run under
rocprofv3 --kernel-trace --stats for the per-kernel split (VCT_K3_PLAN=level: one
lane-per-parent launch per level, for A/B against the block-subtree plan)."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from vct import Context, scenes
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    st = torch.cuda.current_stream()
    ctx.set_stream(st.cuda_stream)
    ctx.voxelize(*scenes.atrium().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR)
    ctx.build_mips()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.reps):
        ctx.build_mips()
    e1.record(st)
    torch.cuda.synchronize()
    print(f"n={a.n} K3 {e0.elapsed_time(e1) / a.reps:.4f} ms per build "
          f"({'per-level' if os.environ.get('VCT_K3_PLAN') == 'level' else 'block subtrees'})")


if __name__ == "__main__":
    main()
