"""How many trace streams: K frames round-robin over S streams (S = 1..4), each frame
waiting for the frame S before it on its stream only, at 1080p on one GPU (by hand, as
vct.multi.FrameTracer would with S buffer sets).  Several stream sets per S, since the
hardware queues a set lands on matter."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def main():
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    n, w, h, frames = 256, 1920, 1080, 60
    world = int(os.environ.get("WORLD", "1"))
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E)
    main_s = torch.cuda.current_stream()
    ctx.set_stream(main_s.cuda_stream)
    ctx.voxelize(*scenes.atrium().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
    ctx.build_mips()
    dev = torch.device("cuda")
    cam = Camera()
    eye = [float(x) for x in cam.position]
    gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)
    from vct.multi import TILE, tiles_for_rank
    npx = tiles_for_rank(w, h, 0, world) * TILE * TILE if world > 1 else w * h
    kw = dict(tile_rank=0, tile_world=world, tile_compact=world > 1)
    outs = [(torch.empty((npx, 4), device=dev), torch.empty((npx, 4), device=dev)) for _ in range(4)]
    for _ in range(40):
        ctx.trace_device(*gb, w, h, eye, outs[0][0], outs[0][1], **kw)
    torch.cuda.synchronize()

    def wall(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3 / frames

    def loop(streams):
        S = len(streams)

        def run():
            for f in range(frames):
                st = streams[f % S]
                st.wait_stream(main_s)
                ctx.set_stream(st.cuda_stream)
                ctx.trace_device(*gb, w, h, eye, outs[f % S][0], outs[f % S][1], **kw)
                ctx.set_stream(main_s.cuda_stream)
                main_s.wait_stream(streams[(f + 1) % S])
            for s_ in streams:
                main_s.wait_stream(s_)
        return run
    print(f"world {world}: one stream {wall(loop([main_s])):.4f} ms/frame", flush=True)
    for S in (2, 3, 4):
        res = []
        for _ in range(3):
            res.append(wall(loop([torch.cuda.Stream() for _ in range(S)])))
        print(f"world {world}: {S} streams " + " ".join(f"{r:.4f}" for r in res), flush=True)


if __name__ == "__main__":
    main()
