"""Host cost of one FrameTracer step (Python + ctypes + HIP launches) on one GPU: a
64x64 frame, whose GPU time is negligible, stepped K times; with and without overlap."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]


def main():
    import torch
    from vct import Context, scenes
    from vct.camera import Camera
    from vct.multi import FrameTracer
    n, w, h, K = 64, 64, 64, 2000
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
    d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
    for _ in range(100):
        ctx.trace_device(*gb, w, h, eye, d, sp)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(K):
        ctx.trace_device(*gb, w, h, eye, d, sp)
    host = (time.perf_counter() - t) / K * 1e6
    torch.cuda.synchronize()
    print(f"trace_device call: {host:.1f} us host", flush=True)
    for ov in (False, True):
        tr = FrameTracer(ctx, torch, None, w, h, 0, 1, dev, overlap=ov)
        for _ in range(100):
            tr.step(gb, eye)
        tr.drain()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(K):
            tr.step(gb, eye)
        host = (time.perf_counter() - t) / K * 1e6
        tr.drain()
        torch.cuda.synchronize()
        print(f"FrameTracer.step overlap={ov}: {host:.1f} us host", flush=True)


if __name__ == "__main__":
    main()
