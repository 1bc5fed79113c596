"""K2 (inject) timing on one GPU: the atrium (or --scene) at n^3, inject `reps` times back
to back; prints ms per inject and a hash of level 0 (variants must agree bit for bit).
VCT_K2_WALK selects the shadow-walk launch (cells per batch * 10000 + block threads)."""
import argparse
import hashlib
import os
import sys

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
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.reps):
        ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    e1.record(st)
    torch.cuda.synchronize()
    h = hashlib.sha256(ctx.download_level(0).tobytes()).hexdigest()[:16]
    print(f"{a.scene} n={a.n} K2 {e0.elapsed_time(e1) / a.reps:.4f} ms per inject "
          f"(VCT_K2_WALK={os.environ.get('VCT_K2_WALK', 'default')}) level0 {h}", flush=True)


if __name__ == "__main__":
    main()
