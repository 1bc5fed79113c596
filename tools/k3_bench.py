"""K3 (mip build) timing on one GPU: a scene at n^3, one build, then build_mips `reps` times
(relight builds: Grid::k3_live; VCT_K3_SPARSE=0 full builds); run under
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
    ap.add_argument("--scene", default="atrium")
    a = ap.parse_args()
    import torch
    from vct import Context, scenes
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E)
    st = torch.cuda.current_stream()
    ctx.set_stream(st.cuda_stream)
    ctx.voxelize(*scenes.SCENES[a.scene]().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR)
    ctx.build_mips()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.reps):
        ctx.build_mips()
    e1.record(st)
    torch.cuda.synchronize()
    sparse = os.environ.get("VCT_K3_SPARSE", "1") != "0"
    print(f"{a.scene} n={a.n} BZ={os.environ.get('VCT_K3_BZ', '4')} K3 {e0.elapsed_time(e1) / a.reps:.4f} ms per build "
          f"({'per-level' if os.environ.get('VCT_K3_PLAN') == 'level' else 'block subtrees'}, "
          f"{'relight builds' if sparse else 'full builds'})")


if __name__ == "__main__":
    main()
