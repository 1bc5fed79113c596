"""Tuner decision log (VCT_TUNE_LOG) over a scene change, and each forced candidate timed (A/B helper)."""
import sys, os, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "voxel-based-global-illumination_amd")]
os.environ["VCT_TUNE_LOG"] = "1"
import torch
from vct import Context, scenes
from vct.camera import Camera
n, w, h = 256, 1920, 1080
g0, E = scenes.grid_for_unit_box(n)
ctx = Context(n, g0, E)
st = torch.cuda.current_stream(); ctx.set_stream(st.cuda_stream)
cam = Camera(); dev = torch.device("cuda")
for name in ("atrium", "courtyard", "atrium"):
    ctx.voxelize(*scenes.SCENES[name]().arrays())
    ctx.inject_directional(scenes.LIGHT_DIR); ctx.build_mips()
    gb = [torch.empty((h, w, 4), device=dev) for _ in range(3)]
    ctx.gbuffer_raster_device(cam, w, h, 0.1, *gb)
    d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
    forms = []
    for i in range(60):
        ctx.trace_device(*gb, w, h, cam.position, d, sp); torch.cuda.synchronize(); forms.append(ctx.trace_form)
    for v in (0x1000000 | 0x4000000, 0x2000000 | 0x4000000, 0x1000000 | 0x8000, 0x2000000 | 0x8000):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3): ctx.trace_device(*gb, w, h, cam.position, d, sp, variant=v)
        e0.record(st)
        for _ in range(10): ctx.trace_device(*gb, w, h, cam.position, d, sp, variant=v)
        e1.record(st); torch.cuda.synchronize()
        print(name, hex(v), round(e0.elapsed_time(e1) / 10, 4), flush=True)
    print(name, "forms", forms, flush=True)
