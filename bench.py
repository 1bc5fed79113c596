#!/usr/bin/env python3
"""bench.py — Mcone-steps/s of the MI355X voxel-cone-tracing pass (BASELINE.json metric).

Workload (BASELINE.json configs[2], the roofline run): 256^3 anisotropic
RGBA32F grid, 1920x1080 G-buffer, 9 diffuse + 1 specular cone.  Sponza is not
available offline, so the scene is the procedural "atrium" stand-in
(vct.scenes.atrium) and the G-buffer is G_scene, rastered by the HIP G-buffer
pass from the reference camera (eye (0,0,3), yaw -90, 45 deg FOV; camera.h:14-18,
assets.cpp:25).  The 1 M-triangle "courtyard" (San Miguel stand-in, curved and
bumpy surfaces) is measured at the same size beside it (`secondary`).

One "step" = one frame of the cone-trace pass (K4) over the whole framebuffer:
each rank traces its interleaved 64x64 tiles (tile t -> rank t % N) and, for
N > 1, the frame is assembled on the presenting rank 0 (every rank sends
exactly its own tiles over RCCL; `--exchange allgather` all-gathers to every
rank instead) and un-permuted there (strong scaling: the frame is fixed, the
tiles are split).  Frames are pipelined as a renderer's frame loop runs them
(vct.multi.FrameTracer): the exchange of frame f overlaps the trace of frame
f+1, and frame f may be traced on trace stream f % 2, so that the next frame's
trace fills the tail of the previous K4 launch -- FrameTracer.tune times both
before the warmup and keeps the faster (`overlap_tune`; `--overlap on|off`
forces it); every timed step still traces, exchanges and un-permutes one
whole frame, and the pipeline is drained inside the timed region.  The
roofline's K4 launch duration (`k4_kernel_ms_avg`) is timed after the loop
with K frames back to back on one stream (the kernel alone; rocprofv3 agrees
with it on a `--overlap off` run, profiles/r03_r3n_ovoff_*); `k4_kernel_ms_avg_overlapped`
is the launches' start-to-end average inside the pipelined loop, where two
traces share the chip, and `roofline.pipelined` the same per-launch work over
the timed loop's time per frame.  The level-0 grid is injected
on rank 0 and broadcast (RCCL) before the timed region, as when the light
changes; every other rank also injects it itself (the replicated alternative,
checked bit-equal); K1/K2/K3, the broadcast, the trace alone (slowest rank) and
the exchange alone are reported beside the metric (K2 and K3 as the mean of 10 calls
queued back to back, with their HBM fractions `k2_roofline` / `k3_roofline`).

value = cone steps of the frame (counted by the kernel; identical to the
oracle's count, tests/test_parity_gpu.py) x K / max-over-ranks wall time.

roofline: K4 is bound by instruction issue, not HBM.  From
the PMC record of the timed K4 form (rocprofv3, profiles/k4_counters.json, valid
only for the library build it was measured on: the file records the .so's
sha256) three rates are formed over the live K4 time -- VALU issue
(SQ_INSTS_VALU against 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction),
scalar issue (SQ_INSTS_SALU against 256 CUs x 2.4 GHz) and the measured HBM
traffic (2 FETCH_SIZE + WRITE_SIZE, gfx950 correction, against 8 TB/s) -- and
`roofline` names the most loaded one (`bound`).  The spec's algorithmic texel
bytes (`gather_bytes`, served ~99 % by LDS / L1 / L2) are reported beside them.
At N > 1 the record is the one of a rank's own launch (`ranksN` keys, measured
by tools/rank_emul.py under rocprofv3).

Beside the metric (rank 0's JSON line): `frame_loop` (N = 1: 5000 default-variant
frames of G_scene and of G_rand after their choice settled: per-frame K4 time and
host launch time, the tuner's hitch check), `multi_config` (BASELINE configs[3]
and [4]: atrium 512^3 at 3840x2160 with 9+1 cones at every N, its 2 GiB level-0
broadcast timed; courtyard 512^3, 16+1 cones, 4K at N = 1 and 8) and, at N > 1
over RCCL, `capi` (one frame assembled through the torch-free C-ABI path,
vct_comm_*: checked bit-equal to the torch frame and timed).

`--gpus N` without WORLD_SIZE in the environment starts the N ranks itself
(one child process per GPU, before anything touches a GPU).  `--dry-run`
rehearses the N-rank plumbing on the CPU (gloo, a pattern-writing stand-in
for the trace; nothing is measured, value = null).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import datetime
import hashlib
import json
import math
import os
import platform
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "voxel-based-global-illumination_amd"))
sys.path.insert(0, REPO)

METRIC = "Mcone-steps/s at 256^3 grid, 1080p, 9 diffuse + 1 spec cone; 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SIMDS, CUS, CLOCK_GHZ = 1024, 256, 2.4
VALU_PEAK_G = SIMDS * CLOCK_GHZ / 2.0      # wave64 VALU instructions / ns: one per 2 cycles per SIMD-32
SALU_PEAK_G = CUS * CLOCK_GHZ              # one scalar instruction per cycle per CU
BYTES_PER_TEXEL = 16       # RGBA32F
BYTES_PER_VALID_PX = 80    # 48 B G-buffer read + 32 B output write
LIB = os.path.join(REPO, "voxel-based-global-illumination_amd", "vct", "libvct_hip.so")
PROFILE = os.path.join(REPO, "profiles", "k4_counters.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--n", type=int, default=256)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--scene", default="atrium")
    p.add_argument("--gbuffer", default="scene", choices=["scene", "rand"])
    p.add_argument("--n-diffuse", type=int, default=9)
    p.add_argument("--no-spec", action="store_true")
    p.add_argument("--variant", type=lambda v: int(v, 0), default=0)
    p.add_argument("--reorder", action="store_true",
                   help="ray reordering (variant bit 0x8000): pixels traced in Morton order of their origin voxel")
    p.add_argument("--exchange", default="present", choices=["present", "allgather"],
                   help="N > 1: assemble the frame on rank 0 (send/recv) or on every rank (all-gather)")
    p.add_argument("--secondary", default="courtyard",
                   help="second scene measured at the same size (empty or 'none': skip)")
    p.add_argument("--stress", default="rand",
                   help="N = 1: also time the cache-hostile G_rand G-buffer on the metric scene, screen "
                        "order vs ray reordering (empty or 'none': skip)")
    p.add_argument("--frame-loop", type=int, default=5000,
                   help="N = 1: frames of the steady-state hitch loop per G-buffer (0: skip)")
    p.add_argument("--multi-config", default="c4,c5",
                   help="BASELINE configs[3] / [4] measured beside the metric (comma list; empty or 'none': skip)")
    p.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                   help="consecutive frames on two trace streams (auto: FrameTracer.tune decides)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--profile-json", default=PROFILE)
    p.add_argument("--dry-run", action="store_true", help="CPU rehearsal of the rank plumbing (gloo), no GPU")
    a = p.parse_args()
    if a.reorder:
        a.variant |= 0x8000
    return a


# ---------------------------------------------------------------------------
# launcher: `--gpus N` without a torch.distributed environment
# ---------------------------------------------------------------------------
def spawn_ranks(args) -> int:
    """Start one child per rank (env RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*) and
    wait; this process never touches a GPU.  Rank 0's stdout is the JSON line."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = None if r == 0 else subprocess.DEVNULL
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out, start_new_session=False))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:     # one rank failed: the others would wait forever in a collective
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


# ---------------------------------------------------------------------------
# roofline inputs
# ---------------------------------------------------------------------------
def lib_sha256() -> str | None:
    try:
        with open(LIB, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def profile_key(n, w, h, scene, gbuffer, nd, spec, variant, world):
    return f"{n}^3 {w}x{h} {scene} G_{gbuffer} {nd}+{1 if spec else 0} v{variant} ranks{world}"


def load_profile(path, key):
    """The PMC record of the timed K4 form for this workload and THIS library build, or (None, reason)."""
    try:
        with open(path) as f:
            prof = json.load(f)
    except (OSError, ValueError) as e:
        return None, f"no profile ({e.__class__.__name__})"
    rec = prof.get(key)
    if rec is None:
        return None, f"no profile entry for '{key}'"
    sha = lib_sha256()
    if rec.get("lib_sha256") != sha:
        return None, "profile measured on another library build"
    return rec, None


def roofline(rec, reason, k4_ms, texels, valid_px, profile_path, key, steps=None):
    """k4_ms None: the record's own rocprofv3 kernel duration is the live time (a line that
    times whole frames only, e.g. `stress`, whose frames include the reorder sort)."""
    if k4_ms is None and rec is not None:
        k4_ms = rec.get("duration_ms")
    gather = texels * BYTES_PER_TEXEL + valid_px * BYTES_PER_VALID_PX if texels is not None else None
    out = {"bound": "issue (VALU)", "achieved": None, "peak": VALU_PEAK_G, "unit": "G VALU wave-instr/s", "frac": None,
           "traffic": None, "gather_bytes": gather,
           "gather_GBs": round(gather / (k4_ms * 1e-3) / 1e9, 1) if gather is not None and k4_ms else None,
           # north_star's "% of HBM roofline": SURVEY 8d's algorithmic bytes over the live K4 time
           # against 8 TB/s.  Above 1 because the gathered texels come from LDS bricks and L2,
           # not HBM (the 60 % HBM target cannot describe an on-chip gather); the
           # counter HBM fraction is "hbm" below, the binding resource "bound"
           "hbm_algorithmic_frac": round(gather / (k4_ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 3)
           if gather is not None and k4_ms else None,
           "texel_fetches_per_launch": texels, "k4_ms": round(k4_ms, 4) if k4_ms else None,
           "peak_basis": "1024 SIMD-32 x 2.4 GHz / 2 cycles per wave64 VALU instruction"}
    if rec is None or not k4_ms:
        out["note"] = reason or "no kernel time"
        return out
    t = k4_ms * 1e-3
    valu, salu = rec["SQ_INSTS_VALU"], rec["SQ_INSTS_SALU"]
    hbm = rec["hbm_bytes_per_launch"]
    v_ach = valu / t / 1e9
    s_ach = salu / t / 1e9
    h_ach = hbm / t / 1e9
    out.update({
        "achieved": round(v_ach, 1), "frac": round(v_ach / VALU_PEAK_G, 4), "traffic": hbm,
        "valu_insts_per_launch": valu,
        "salu": {"achieved": round(s_ach, 1), "peak": SALU_PEAK_G, "unit": "G SALU instr/s",
                 "frac": round(s_ach / SALU_PEAK_G, 4), "insts_per_launch": salu},
        "hbm": {"achieved": round(h_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(h_ach / HBM_PEAK_GBS, 4)},
        "profile": f"{os.path.relpath(profile_path, REPO)}#{key}",
        "profile_kernel_ms": rec.get("duration_ms"),
        "profile_tag": rec.get("tag"),
    })
    if steps:
        # wave instructions per cone step (a wave-step advances ~62 lanes' cone steps)
        out["valu_per_cone_step"] = round(valu / steps, 3)
        out["salu_per_cone_step"] = round(salu / steps, 3)
    if rec.get("effective_clock_ghz"):
        # the chip runs below the 2.4 GHz the peak assumes (DVFS under load); the VALU
        # fraction against the issue rate at the clock measured on the profiled dispatches
        ghz = rec["effective_clock_ghz"]
        out["effective_clock_ghz"] = round(ghz, 3)
        out["valu_frac_at_measured_clock"] = round(v_ach / (1024 * ghz / 2), 4)
    if rec.get("SQ_WAVE_CYCLES"):
        # fraction of wave cycles in which the wave issued (the rest: waits and issue stalls)
        out["issue_active"] = round(rec["SQ_ACTIVE_INST_ANY"] / rec["SQ_WAVE_CYCLES"], 4)
        out["wait_any"] = round(rec["SQ_WAIT_ANY"] / rec["SQ_WAVE_CYCLES"], 4)
    out["valu"] = {"achieved": out["achieved"], "peak": VALU_PEAK_G, "unit": out["unit"], "frac": out["frac"]}
    # name the resource that binds: the most loaded of VALU issue, scalar issue and HBM
    if out["salu"]["frac"] > max(out["frac"], out["hbm"]["frac"]):
        out.update({"bound": "issue (scalar)", "achieved": out["salu"]["achieved"], "peak": SALU_PEAK_G,
                    "unit": "G SALU instr/s", "frac": out["salu"]["frac"],
                    "peak_basis": "256 CUs x 2.4 GHz x one scalar instruction per cycle per CU"})
    elif out["hbm"]["frac"] > out["frac"]:
        out.update({"bound": "hbm", "achieved": round(h_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": out["hbm"]["frac"], "peak_basis": "HBM3E 8 TB/s spec"})
    return out


# ---------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the C oracle on a bounded sample of the same frame
# ---------------------------------------------------------------------------
def host_info():
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    model = platform.processor() or None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    quota, raw = cgroup_cpus()
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": int(omp) if omp and omp.isdigit() else None,
            "cgroup_cpu_max": raw, "cgroup_cpus": quota}


def cgroup_cpus():
    """CPUs the job's cgroup may use: cgroup v2 cpu.max (quota period) or v1
    cfs_quota_us / cfs_period_us; (None, raw) when there is no quota."""
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.max"):
        try:
            raw = open(path).read().strip()
        except OSError:
            continue
        q, _, per = raw.partition(" ")
        if q == "max" or not per:
            return None, raw
        return max(1, math.ceil(int(q) / int(per))), raw
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        raw = f"cfs_quota_us={q} cfs_period_us={per}"
        return (max(1, math.ceil(q / per)) if q > 0 else None), raw
    except (OSError, ValueError):
        return None, None


def cpu_share(host):
    """Threads for the CPU baseline and why: the cgroup quota if there is one (capped by
    the affinity mask); else the pool's documented per-GPU share, which the pool exports
    as OMP_NUM_THREADS (16 per GPU on the MI355X boxes, whose affinity mask and
    os.cpu_count() show the whole machine); else the affinity mask."""
    aff = host["affinity_cpus"] or os.cpu_count() or 1
    if host["cgroup_cpus"]:
        return min(host["cgroup_cpus"], aff), f"cgroup quota {host['cgroup_cpu_max']}"
    if host["omp_num_threads"]:
        return min(host["omp_num_threads"], aff), (
            f"no cgroup CPU quota ({host['cgroup_cpu_max'] or 'cpu.max absent'}); the GPU pool's per-GPU CPU "
            f"share, exported as OMP_NUM_THREADS={host['omp_num_threads']} (the affinity mask lists {aff})")
    return aff, "affinity mask (no cgroup quota, no OMP_NUM_THREADS)"


def cpu_baseline(ctx, n, g0, E, gb_host, eye, n_diffuse, spec, steps_px_gpu, target_s):
    import numpy as np
    from oracle import oracle as O
    O.build()
    pos, nrm, alb = gb_host
    h, w = pos.shape[:2]
    r0 = ctx.download_level(0)
    parts = []
    for l in range(1, ctx.num_levels):
        for f in range(ctx.level_dims(l)[1]):
            parts.append(ctx.download_level(l, f).ravel())
    pyr = np.concatenate(parts)
    host = host_info()
    cores, basis = cpu_share(host)
    host["cores_basis"] = basis
    probe_step = 128
    t0 = time.perf_counter()
    O.trace(n, g0, E, r0, pyr, pos, nrm, alb, eye, aniso=True, n_diffuse=n_diffuse, specular=spec,
            row_step=probe_step, threads=cores)
    tp = max(time.perf_counter() - t0, 1e-3)
    rows_probe = len(range(0, h, probe_step))
    rows_target = max(1, int(rows_probe * target_s / tp))
    row_step = max(1, h // rows_target)
    t0 = time.perf_counter()
    res = O.trace(n, g0, E, r0, pyr, pos, nrm, alb, eye, aniso=True, n_diffuse=n_diffuse, specular=spec,
                  row_step=row_step, threads=cores)
    dt = time.perf_counter() - t0
    rows = list(range(0, h, row_step))
    match = bool(np.array_equal(res["steps_px"][rows], steps_px_gpu[rows]))
    steps, reps = res["cone_steps"], 1
    if row_step == 1 and dt < 0.5 * target_s:
        # the whole frame takes less than the target: time repeated whole frames instead
        reps = min(50, max(1, int(math.ceil(target_s / max(dt, 1e-3)))))
        t0 = time.perf_counter()
        for _ in range(reps):
            O.trace(n, g0, E, r0, pyr, pos, nrm, alb, eye, aniso=True, n_diffuse=n_diffuse, specular=spec,
                    row_step=1, threads=cores)
        dt = time.perf_counter() - t0
        steps *= reps
    sample = (f"whole frame x {reps} ({res['cone_steps']} cone steps each, {dt:.1f} s)" if row_step == 1 else
              f"rows y % {row_step} == 0 ({len(rows)} of {h} rows, {res['cone_steps']} cone steps, {dt:.1f} s)")
    return {
        "value": steps / dt / 1e6,
        "unit": "Mcone-steps/s",
        "cores": cores,
        "kind": "port",
        "sample": sample + "; C oracle -O3 x86-64-v3 OpenMP, one thread per core used",
        "steps_match_gpu": match,
        "host": host,
    }


# what each procedural scene stands in for (the reference's assets are not available offline)
STAND_IN = {"atrium": " (Sponza stand-in)", "courtyard": " (San Miguel stand-in)"}


def max_over_ranks(torch, dist, dev, vals, world):
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


_T0 = time.perf_counter()


def progress(rank, what):
    """one line per phase on stderr (rank 0): a long run keeps writing while it works"""
    if rank == 0:
        print(f"[bench {time.perf_counter() - _T0:7.1f} s] {what}", file=sys.stderr, flush=True)


_JSON_FD = None


def protect_stdout():
    """The JSON line is the only thing on stdout: native libraries of a rank (gloo's
    connection message, RCCL) print to fd 1 too, so fd 1 becomes stderr and the line
    goes to the saved descriptor."""
    global _JSON_FD
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)


def emit(obj):
    line = json.dumps(obj) + "\n"
    if _JSON_FD is None:
        sys.stdout.write(line)
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line.encode())


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world == 0:
        if args.gpus > 1:
            sys.exit(spawn_ranks(args))     # before anything touches a GPU
        world = 1
    if args.gpus != world:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE is {world}: one process per GPU")
    protect_stdout()
    if args.dry_run:
        return dry_run(args, world)
    run(args, world)


def dry_run(args, world):
    """The N-rank plumbing on the CPU: gloo process group, the FrameTracer exchange in the
    chosen mode with a pattern-writing stand-in trace, max-over-ranks timing, one JSON
    line.  Checks the assembled frame exactly; measures nothing."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from vct.multi import FrameTracer, PatternContext
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    w, h = args.width, args.height
    dev = torch.device("cpu")
    res = {}
    for mode in ("present", "allgather"):
        tr = FrameTracer(PatternContext(torch), torch, dist, w, h, rank, world, dev, mode=mode)
        gb = (None, None, None)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tr.step(gb, (0.0, 0.0, 3.0))
        tr.drain()
        el = max_over_ranks(torch, dist, dev, [time.perf_counter() - t0], world)[0]
        ok = True
        if tr.holds_frame:
            ref = np.arange(w * h, dtype=np.float32).reshape(h, w, 1).repeat(4, 2)
            ok = np.array_equal(tr.diff.numpy(), ref) and np.array_equal(tr.spec.numpy(), -ref)
        ok = max_over_ranks(torch, dist, dev, [0.0 if ok else 1.0], world)[0] == 0.0
        res[mode] = {"frame_ok": ok, "ms_per_step": round(el / args.steps * 1e3, 3)}
    if rank == 0:
        emit({
            "metric": METRIC, "value": None, "unit": "Mcone-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "data": "dry run (CPU, gloo, pattern stand-in trace)",
            "dry_run": True, "exchange": args.exchange, "exchange_check": res,
            "config": {"workload": "rank plumbing only", "width": w, "height": h,
                       "parallelism": f"screen-tiles x{world}"},
            "trace_ms_max_rank": None, "gather_ms": None, "allgather_ms": None,
        })
    if world > 1:
        dist.destroy_process_group()


_SCENES = {}


def scene_arrays(name):
    """vct.scenes arrays, built once per process (the 1 M-triangle courtyard takes seconds)"""
    if name not in _SCENES:
        from vct import scenes
        _SCENES[name] = scenes.SCENES[name]().arrays()
    return _SCENES[name]


ATOMIC_PEAK_GBS = 1300.0   # chip-wide atomic rate (MI355X_MICROARCH.md 'Global float atomics')
RELIGHT_PROFILE = os.path.join(REPO, "profiles", "relight_counters.json")


def load_relight_profile(n, scene):
    """The rocprofv3 records of K1 / K2 / K3 for this grid and scene and THIS library build
    (tools/pmc_all.sh -> profiles/relight_counters.json), or (None, reason)."""
    try:
        with open(RELIGHT_PROFILE) as f:
            db = json.load(f)
    except (OSError, ValueError) as e:
        return None, f"no relight profile ({e.__class__.__name__})"
    rec = db.get(f"{n}^3 {scene}")
    if rec is None:
        return None, f"no relight profile entry for '{n}^3 {scene}'"
    if any(v.get("lib_sha256") != lib_sha256() for v in rec.values()):
        return None, "relight profile measured on another library build"
    return rec, None


def k3_relight_bytes(ao_alpha, n):
    """Algorithmic bytes of a relight K3 build (Grid::k3_live, vct_mips.hip): the first
    launch reads level 0 and writes levels 1..3 only for its blocks of 16 x 16 x 2 BZ
    level-0 voxels that hold an occupied voxel (BZ = VCT_K3_BZ, 4 by default); the later
    launches read level 3 and write levels 4..L whole.  -> (bytes, live block fraction)"""
    import numpy as np
    L = int(math.log2(n))
    bz = int(os.environ.get("VCT_K3_BZ", "4"))
    bz = bz if bz in (2, 8) else 4
    occ = ao_alpha > 0                                  # [z][y][x]
    zb = 2 * bz
    live = occ.reshape(n // zb, zb, n // 16, 16, n // 16, 16).any(axis=(1, 3, 5))
    frac = float(live.mean())
    top = min(3, L)
    first = n ** 3 * 16 + sum(6 * (n >> l) ** 3 * 16 for l in range(1, top + 1))
    rest = (6 * (n >> top) ** 3 * 16 + sum(6 * (n >> l) ** 3 * 16 for l in range(top + 1, L + 1))) if L > top else 0
    return int(frac * first + rest), frac


def relight_roofline(ctx, n, scene, k1_ms, k2_ms, k3_ms, k3_sparse=False):
    """Rooflines of the relight kernels.  From the rocprofv3 record of this build (per call:
    VALU wave-instructions, HBM bytes = (2 FETCH_SIZE + WRITE_SIZE) x 1024 and, for K1, the
    L2's atomic requests x 64 B) three rates are formed over the stage's kernel time --
    VALU issue (1 228.8 G/s), HBM (8 TB/s), atomics (K1 only, 1.3 TB/s) -- and `bound`
    names the most loaded.  K2 / K3 use the bench's own time (10 calls queued back to
    back); K1's host-timed call includes a host read-back of its candidate count, so its
    rates use the record's summed kernel durations (`kernel_ms`).  The algorithmic bytes
     stay beside them: K3 reads level 0 once and writes every face of levels
    1..L; K2 reads the albedo / normal of every occupied voxel (32 B) and writes its
    level-0 texel (16 B)."""
    import numpy as np
    L = int(math.log2(n))
    k3_bytes = n ** 3 * 16 + sum(6 * (n >> l) ** 3 * 16 for l in range(1, L + 1))
    ao, _ = ctx.download_voxels()
    k3_live = None
    if k3_sparse and n >= 16 and os.environ.get("VCT_K3_SPARSE", "1") != "0":
        # a relight build skips K3's blocks without an occupied voxel: count only the rest
        k3_bytes, k3_live = k3_relight_bytes(ao[..., 3], n)
    occ = int(np.count_nonzero(ao[..., 3] > 0))
    k2_bytes = occ * 48
    rec, reason = load_relight_profile(n, scene)
    out = {}
    for name, alg, ms in (("k1", None, k1_ms), ("k2", k2_bytes, k2_ms), ("k3", k3_bytes, k3_ms)):
        r = {"bytes": alg, "bench_ms": round(ms, 4) if ms else None}
        if alg is not None and ms:
            gbs = alg / (ms * 1e-3) / 1e9
            r["algorithmic_GBs"] = round(gbs, 1)
            r["algorithmic_frac"] = round(gbs / HBM_PEAK_GBS, 4)
        st = (rec or {}).get(name)
        if st is None:
            r.update({"bound": None, "frac": None, "note": reason or f"no {name} record"})
            out[f"{name}_roofline"] = r
            continue
        t_ms = st["kernel_ms_per_call"] if name == "k1" else ms
        t = t_ms * 1e-3
        rates = {"issue (VALU)": (st.get("SQ_INSTS_VALU", 0) / t / 1e9, VALU_PEAK_G, "G VALU wave-instr/s"),
                 "hbm": (st.get("hbm_bytes_per_call", 0) / t / 1e9, HBM_PEAK_GBS, "GB/s")}
        if name == "k1":
            rates["atomics"] = (st.get("atomic_bytes_per_call", 0) / t / 1e9, ATOMIC_PEAK_GBS, "GB/s")
        bound = max(rates, key=lambda k_: rates[k_][0] / rates[k_][1])
        ach, peak, unit = rates[bound]
        r.update({"bound": bound, "achieved": round(ach, 1), "peak": peak, "unit": unit,
                  "frac": round(ach / peak, 4), "kernel_ms": round(t_ms, 4),
                  "rates": {k_: {"achieved": round(v[0], 1), "peak": v[1], "unit": v[2], "frac": round(v[0] / v[1], 4)}
                            for k_, v in rates.items()},
                  "traffic": st.get("hbm_bytes_per_call"), "l2_hit_rate": round(st.get("l2_hit_rate", 0.0), 4),
                  "wait_any": round(st.get("wait_any", 0.0), 4), "issue_active": round(st.get("issue_active", 0.0), 4),
                  "kernels": st.get("kernels"), "profile": f"profiles/relight_counters.json#{n}^3 {scene}",
                  "profile_tag": st.get("tag")})
        out[f"{name}_roofline"] = r
    out["k2_roofline"]["occupied_voxels"] = occ
    out["k3_roofline"]["build"] = ("relight (K2 level 0, same occupancy: blocks without an occupied voxel "
                                   "and the K4 maps skipped)" if k3_live is not None else "full")
    if k3_live is not None:
        out["k3_roofline"]["live_block_frac"] = round(k3_live, 4)
    return out


def measure_scene(args, torch, dist, ctx, scene_name, rank, world, dev, stream, counting_only=False,
                  relight_roofs=False):
    """K1-K3 for `scene_name`, the G-buffer, one counting frame, then K timed frames."""
    import numpy as np
    from vct import scenes
    from vct.camera import Camera
    from vct.multi import FrameTracer, compact_index
    n, w, h = args.n, args.width, args.height

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    def timed_queued(fn, reps=10):
        """ms per call of `reps` calls queued back to back on the stream (HIP events): the
        relight kernels as a frame runs them, without a host round trip per call"""
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    v, i, m, k = scene_arrays(scene_name)
    # K1 on every rank (each process holds the scene, as the reference's loader does),
    # from device-resident geometry (the reference's meshes live in GL buffers);
    # K1-K3 are timed on a second call (the first one allocates their scratch)
    dgeo = (torch.from_numpy(v).to(dev), torch.from_numpy(i.astype(np.int32)).to(dev),
            torch.from_numpy(m.astype(np.int32)).to(dev), torch.from_numpy(k).to(dev))
    ctx.voxelize_device(*dgeo)
    r = {"k1_voxelize_ms": round(timed(lambda: ctx.voxelize_device(*dgeo)), 3)}
    del dgeo
    level0 = torch.empty((n ** 3 * 4,), dtype=torch.float32, device=dev)
    k2_ms = 0.0
    if rank == 0:
        ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
        k2_ms = timed_queued(lambda: ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR))
        ctx.copy_level0_to_device(level0)
    bcast_ms, k2_rep_ms, k2_rep_match = 0.0, k2_ms, True
    if world > 1:
        dist.barrier()
        bcast_ms = timed(lambda: dist.broadcast(level0, src=0))
        # SURVEY 8e alternative to the broadcast: every rank runs K2 itself (K2 is
        # deterministic, so the replicated grid must equal the broadcast one bit for bit)
        if rank != 0:
            ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
            k2_rep_ms = timed_queued(lambda: ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR))
            mine = torch.empty_like(level0)
            ctx.copy_level0_to_device(mine)
            k2_rep_match = bool(torch.equal(mine, level0))
            del mine
        k2_rep_ms, mism = max_over_ranks(torch, dist, dev, [k2_rep_ms, 0.0 if k2_rep_match else 1.0], world)
        k2_rep_match = mism == 0.0
        ctx.set_level0_from_device(level0)
    del level0
    ctx.build_mips()
    k3_ms = timed_queued(ctx.build_mips)
    # world 1: level 0 came from K2, so those were relight builds (Grid::k3_live).  With more
    # ranks the broadcast level 0 is a dense write (full builds); the replicated-K2 frame
    # (every rank injects itself) gets relight builds: timed here after a local injection
    # (level 0 equals the broadcast one bit for bit, replicated_k2_equals_bcast)
    k3_rep_ms = k3_ms
    if world > 1:
        ctx.inject_directional(scenes.LIGHT_DIR, scenes.LIGHT_COLOR)
        ctx.build_mips()
        k3_rep_ms = max_over_ranks(torch, dist, dev, [timed_queued(ctx.build_mips)], world)[0]
    r.update({"k2_inject_ms": round(k2_ms, 3), "k3_mips_ms": round(k3_ms, 3), "grid_bcast_ms": round(bcast_ms, 3),
              "k3_mips_relight_ms": round(k3_rep_ms, 3)})
    if relight_roofs:
        # world 1: level 0 comes from K2 here, so the timed builds are relight builds; with
        # more ranks it arrived through set_level0_from_device (a dense write: full builds)
        r.update(relight_roofline(ctx, n, scene_name, r["k1_voxelize_ms"], k2_ms, k3_ms, k3_sparse=world == 1))

    progress(rank, f"  {scene_name}: K1-K3 timed")
    cam = Camera()
    eye = [float(x) for x in cam.position]
    if args.gbuffer == "scene":
        gb = tuple(torch.empty((h, w, 4), dtype=torch.float32, device=dev) for _ in range(3))
        ctx.gbuffer_raster_device(cam, w, h, scenes.ROUGHNESS, *gb)   # row f2, == the ray caster
    else:
        ao, nm = ctx.download_voxels()
        host = scenes.gbuffer_rand(ao, nm, ctx.aabb_min, ctx.extent, w, h, seed=42)
        gb = tuple(torch.from_numpy(a).to(dev) for a in host)
    torch.cuda.synchronize()

    tracer = FrameTracer(ctx, torch, dist, w, h, rank, world, dev, mode=args.exchange,
                         overlap={"auto": None, "on": True, "off": False}[args.overlap])
    # counting pass (same kernel, counters on): frame cone steps and texel fetches
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    steps_px = torch.zeros((h, w), dtype=torch.int32, device=dev)
    tracer.trace_local(gb, eye, cone_steps=cnt[0:1], texel_fetches=cnt[1:2], steps_px=steps_px,
                       variant=args.variant)
    torch.cuda.synchronize()
    local_steps, local_texels = int(cnt[0].item()), int(cnt[1].item())
    # the counting frame's planes: the timed frames (another compiled form, no counters,
    # perhaps reordered or dispatched longest first) must equal them bit for bit
    lp = tracer.local_planes(0)
    counted = None if lp is None else (lp[0].clone(), lp[1].clone())
    valid = (gb[0][..., 3] != 0).reshape(-1).cpu().numpy()
    fi, _ = compact_index(w, h, rank, world)
    local_valid = int(valid[fi].sum())
    tot = torch.tensor([local_steps, local_valid], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
    frame_steps, frame_valid = int(tot[0].item()), int(tot[1].item())

    # the context times the two compiled forms of K4 on its first counter-free launches of a
    # workload and keeps the faster (vct_trace_form); let that settle before the warmup
    r["k4_form"] = settle_form(ctx, torch, lambda: tracer.trace_local(gb, eye, variant=args.variant))
    # one stream or two (FrameTracer.tune: 16 + 16 timed frames, before the warmup)
    progress(rank, f"  {scene_name}: counting frame done")
    r["overlap_tune"] = tracer.tune(gb, eye, variant=args.variant) if tracer.auto else None
    progress(rank, f"  {scene_name}: overlap tuned")
    for _ in range(args.warmup):
        tracer.frame(gb, eye, variant=args.variant)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        tracer.step(gb, eye, variant=args.variant, events=ev[s])
    tracer.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(torch, dist, dev, [elapsed], world)[0]
    progress(rank, f"  {scene_name}: {args.steps} timed frames done")
    lp = tracer.local_planes(tracer.last_buf)       # the last timed frame (drained above)
    last = None if lp is None else (lp[0].clone(), lp[1].clone())   # compared after the K4-alone loop
    k4_ov_ms = [a.elapsed_time(b) for a, b in ev]
    # K4 alone (the roofline's launch duration): K frames back to back on the ctx stream,
    # no other work on the GPU -- in the pipelined loop consecutive traces share the chip.
    # They run the candidate settled before the warmup (r["k4_form"], the one the PMC record
    # describes), forced: after overlapped frames the tuner may be re-timing its candidates
    # (its samples are taken on one stream), and a launch of the timing would be of another
    # form.  Forcing changes the arithmetic of nothing (every candidate is bit-identical).
    alone_v = args.variant
    if r["k4_form"] is not None and r["k4_form"] >= 0 and (args.variant & 0xff) == 0:
        f = r["k4_form"]
        alone_v = (args.variant & ~0x7008000) | (0x2000000 if f & 1 else 0x1000000) | (0x8000 if f & 2 else 0x4000000)
    tracer.trace_local(gb, eye, variant=alone_v)        # the forced workload's first launch (code load)
    iev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    for s in range(args.steps):
        iev[s][0].record(stream)
        tracer.trace_local(gb, eye, variant=alone_v)
        iev[s][1].record(stream)
    torch.cuda.synchronize()
    r["k4_form_alone"] = ctx.trace_form
    k4_ms = [a.elapsed_time(b) for a, b in iev]
    same = counted is None or (torch.equal(last[0], counted[0]) and torch.equal(last[1], counted[1]))
    timed_equals_counting = max_over_ranks(torch, dist, dev, [0.0 if same else 1.0], world)[0] == 0.0
    del counted, last
    k4_avg_ms = sum(k4_ms) / len(k4_ms)
    k4_med_ms = sorted(k4_ms)[len(k4_ms) // 2]
    ms_per_step = elapsed / args.steps * 1e3
    r.update({
        "value": frame_steps * args.steps / elapsed / 1e6, "ms_per_step": ms_per_step, "frame_cone_steps": frame_steps,
        "valid_px": frame_valid, "k4_kernel_ms_avg": k4_avg_ms, "k4_kernel_ms_median": k4_med_ms,
        "k4_kernel_ms_avg_overlapped": sum(k4_ov_ms) / len(k4_ov_ms), "overlap": tracer.overlap,
        "k4_kernel_ms_min": min(k4_ms), "k4_kernel_ms_max": max(k4_ms),
        "local_texels": local_texels, "local_valid": local_valid, "local_steps": local_steps,
        "frame_relight_ms": round(min(k2_ms + bcast_ms + k3_ms, k2_rep_ms + k3_rep_ms) + ms_per_step, 3),
        "frame_relight_bcast_ms": round(k2_ms + bcast_ms + k3_ms + ms_per_step, 3),
        "frame_relight_replicated_ms": round(k2_rep_ms + k3_rep_ms + ms_per_step, 3),
        "replicated_k2_equals_bcast": k2_rep_match, "timed_equals_counting": timed_equals_counting,
        "_gb": gb, "_eye": eye, "_steps_px": steps_px,
    })
    if world > 1:
        # the parts of a step alone (not overlapped): the slowest rank's trace, and each
        # exchange form (RCCL send/recv to rank 0; all-gather to every rank) + its untile
        r["trace_ms_max_rank"] = round(max_over_ranks(torch, dist, dev, [k4_avg_ms], world)[0], 4)
        for mode, key in (("present", "gather_ms"), ("allgather", "allgather_ms")):
            tx = tracer if mode == args.exchange else FrameTracer(ctx, torch, dist, w, h, rank, world, dev, mode=mode)
            tx.trace_local(gb, eye, variant=args.variant)
            tx.gather()
            gev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.steps)]
            dist.barrier()
            torch.cuda.synchronize()
            for s in range(args.steps):
                gev[s][0].record(stream)
                tx.gather()
                gev[s][1].record(stream)
            torch.cuda.synchronize()
            g_ms = sum(a.elapsed_time(b) for a, b in gev) / args.steps
            r[key] = round(max_over_ranks(torch, dist, dev, [g_ms], world)[0], 4)
            del tx
    return r


def form_name(f):
    """vct_trace_form -> its description (None while timing)"""
    if f is None or f < 0:
        return None
    return ("occupancy, 5 waves/SIMD" if f & 1 else "union (bricks of up to six faces), 4 waves/SIMD") + (
        ", ray reordering" if f & 2 else ", screen order")


def settle_form(ctx, torch, launch, stable=24, max_launches=256):
    """Launch (one frame at a time) until the context's choice for this workload has held
    for `stable` launches -- also when a choice made on another G-buffer or scene under
    the same workload key is first re-timed by the drift watch; returns it."""
    last, run = None, 0
    for _ in range(max_launches):
        launch()
        torch.cuda.synchronize()
        f = ctx.trace_form
        run = run + 1 if (f >= 0 and f == last) else 0
        last = f
        if run >= stable:
            break
    return ctx.trace_form


def frame_loop(torch, ctx, gb, w, h, eye, stream, frames, variant=0):
    """A renderer's steady state: `frames` default-variant frames on one G-buffer after
    the context's choice for it has settled.  Per frame: the K4 time on the stream
    (events) and the host time of the trace call (a launch path that blocked on the GPU
    would show here).  The tuner watches every 2nd launch without blocking and times
    again only on a drift (vct_trace_form), so max / median stays near 1."""
    import numpy as np
    d, sp = torch.empty((h, w, 4), device=gb[0].device), torch.empty((h, w, 4), device=gb[0].device)
    launch = lambda: ctx.trace_device(*gb, w, h, eye, d, sp, variant=variant)   # noqa: E731
    settled = settle_form(ctx, torch, launch)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(frames)]
    host = np.empty(frames)
    forms = set()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(frames):         # one frame in flight, as a renderer presents each frame
        ev[i][0].record(stream)
        t = time.perf_counter()
        launch()
        host[i] = time.perf_counter() - t
        ev[i][1].record(stream)
        ev[i][1].synchronize()
        if i % 250 == 0:
            forms.add(ctx.trace_form)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    forms.add(ctx.trace_form)
    ms = np.array([a.elapsed_time(b) for a, b in ev])
    med = float(np.median(ms))
    return {"frames": frames, "settled_form": form_name(settled), "k4_ms_median": round(med, 4),
            "k4_ms_p99": round(float(np.percentile(ms, 99)), 4),
            "k4_ms_p999": round(float(np.percentile(ms, 99.9)), 4), "k4_ms_max": round(float(ms.max()), 4),
            "max_over_median": round(float(ms.max()) / med, 3),
            # isolated spikes (a single slow frame in 5 000 with no tuner activity: the tuner
            # logs every re-timing under VCT_TUNE_LOG) show up here as a count of 1-2
            "frames_over_1p5x_median": int((ms > 1.5 * med).sum()),
            "host_launch_ms_median": round(float(np.median(host)) * 1e3, 4),
            "host_launch_ms_max": round(float(host.max()) * 1e3, 4), "wall_ms_per_frame": round(wall / frames * 1e3, 4),
            "forms_seen": sorted(form_name(f) or "timing" for f in forms)}


MULTI_CONFIGS = {
    # BASELINE.json configs[3]: "Sponza, 512^3 grid, 4K framebuffer, screen tiles across 2/4/8 MI355X with RCCL grid bcast"
    "c4": {"scene": "atrium", "n": 512, "width": 3840, "height": 2160, "n_diffuse": 9, "ranks": None},
    # configs[4]: "San Miguel, 512^3 6-face anisotropic grid, 16 cones, 4K, 8 MI355X" (+ one GPU for the curve)
    "c5": {"scene": "courtyard", "n": 512, "width": 3840, "height": 2160, "n_diffuse": 16, "ranks": (1, 8)},
}


def measure_config(args, torch, dist, rank, world, dev, stream, cfg):
    """One BASELINE configuration beside the metric: its own context, K1-K3, the level-0
    broadcast (N > 1, timed), the pipelined frame loop, the slowest rank's trace."""
    import copy
    from vct import Context, scenes
    a = copy.copy(args)
    a.n, a.width, a.height, a.n_diffuse, a.gbuffer = cfg["n"], cfg["width"], cfg["height"], cfg["n_diffuse"], "scene"
    g0, E = scenes.grid_for_unit_box(a.n)
    ctx = Context(a.n, g0, E, aniso=True, n_diffuse=a.n_diffuse, specular=not args.no_spec, device=dev.index)
    ctx.set_stream(stream.cuda_stream)
    m = measure_scene(a, torch, dist, ctx, cfg["scene"], rank, world, dev, stream)
    key = profile_key(a.n, a.width, a.height, cfg["scene"], "scene", a.n_diffuse, not args.no_spec, args.variant, world)
    roof = roofline(*load_profile(args.profile_json, key), m["k4_kernel_ms_avg"], m["local_texels"], m["local_valid"],
                    args.profile_json, key, steps=m["local_steps"])
    out = {"workload": f"{cfg['scene']}{STAND_IN.get(cfg['scene'], '')}, {a.n}^3 aniso RGBA32F, "
                       f"{a.width}x{a.height}, {a.n_diffuse}+{0 if args.no_spec else 1} cones",
           "value": round(m["value"], 2), "unit": "Mcone-steps/s", "ms_per_step": round(m["ms_per_step"], 4),
           "frame_cone_steps": m["frame_cone_steps"], "k4_kernel_ms_avg_rank0": round(m["k4_kernel_ms_avg"], 4),
           "k4_form_rank0": form_name(m["k4_form"]), "overlap_tune_rank0": m["overlap_tune"],
           "value_single_launch": round(m["frame_cone_steps"] / m["k4_kernel_ms_avg"] / 1e3, 2) if world == 1 else None,
           "roofline_rank0": roof}
    for k_ in ("timed_equals_counting", "k1_voxelize_ms", "k2_inject_ms", "k3_mips_ms", "k3_mips_relight_ms",
               "grid_bcast_ms", "frame_relight_ms", "replicated_k2_equals_bcast", "trace_ms_max_rank", "gather_ms",
               "allgather_ms"):
        if k_ in m:
            out[k_] = m[k_]
    if world > 1:
        out["grid_bcast_GBs"] = round(a.n ** 3 * 16 / (m["grid_bcast_ms"] * 1e-3) / 1e9, 1) if m["grid_bcast_ms"] else None
    del m
    ctx.close()
    torch.cuda.empty_cache()
    return out


def capi_leg(args, torch, dist, ctx, rank, world, dev, stream, gb, eye):
    """N > 1 over RCCL: the torch-free C-ABI path (include/vct.h vct_comm_*, the one a
    C++ host started once per GPU uses).  The ncclUniqueId goes from rank 0 to every
    rank over the torch group (vct.multi.share_comm_id); level 0 is broadcast in place
    (vct_comm_broadcast_level0, must leave the grid unchanged: every rank already holds
    it); one frame is assembled on rank 0 (root 0: ncclSend/ncclRecv of packed tiles)
    and on every rank (VCT_ALL_RANKS: one ncclAllGather), each checked bit-equal to the
    torch FrameTracer's frame and timed over `steps` synchronous frames."""
    from vct import VCT_ALL_RANKS
    from vct.multi import FrameTracer, share_comm_id
    w, h = args.width, args.height
    ref = FrameTracer(ctx, torch, dist, w, h, rank, world, dev, mode="allgather")
    ref_d, ref_s = ref.frame(gb, eye, variant=args.variant)
    torch.cuda.synchronize()
    cid = share_comm_id(dist, rank)
    ctx.comm_set_timeout(120000)
    ctx.comm_init(cid, world, rank)
    c_rank, c_n = ctx.comm_rank()           # what the RCCL communicator itself holds
    ok_ranks = max_over_ranks(torch, dist, dev, [0.0 if (c_rank, c_n) == (rank, world) else 1.0], world)[0] == 0.0
    n = ctx.n
    before = torch.empty((n ** 3 * 4,), dtype=torch.float32, device=dev)
    after = torch.empty_like(before)
    ctx.copy_level0_to_device(before)
    dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    ctx.comm_broadcast_level0(0)
    ctx.comm_synchronize()
    bcast_ms = (time.perf_counter() - t) * 1e3
    ctx.copy_level0_to_device(after)
    torch.cuda.synchronize()
    bcast_ok = bool(torch.equal(before, after))
    del before, after
    ctx.build_mips()
    out = {"bcast_equal": bcast_ok, "vct_comm_nranks": c_n, "vct_comm_ranks_match": ok_ranks}
    d, sp = torch.empty((h, w, 4), device=dev), torch.empty((h, w, 4), device=dev)
    for root, name in ((0, "present"), (VCT_ALL_RANKS, "allgather")):
        d.fill_(-1.0)
        sp.fill_(-1.0)
        ctx.comm_trace_frame(*gb, w, h, eye, d, sp, root=root, variant=args.variant)
        ctx.comm_synchronize()
        ok = True
        if root == VCT_ALL_RANKS or rank == root:
            ok = bool(torch.equal(d, ref_d) and torch.equal(sp, ref_s))
        dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            ctx.comm_trace_frame(*gb, w, h, eye, d, sp, root=root, variant=args.variant)
        ctx.comm_synchronize()
        ms = (time.perf_counter() - t) / args.steps * 1e3
        bad, ms = max_over_ranks(torch, dist, dev, [0.0 if ok else 1.0, ms], world)
        out[f"{name}_equal"] = bad == 0.0
        out[f"{name}_frame_ms"] = round(ms, 4)
    bad = max_over_ranks(torch, dist, dev, [0.0 if bcast_ok else 1.0, bcast_ms], world)
    out["bcast_equal"], out["bcast_ms"] = bad[0] == 0.0, round(bad[1], 3)
    ctx.comm_destroy()
    return out


def stress_rand(args, torch, ctx, dev, stream):
    """G_rand (independent random surface points and normals per pixel) on the
    scene in `ctx`: the K4 pass in screen order (0x4000000), with ray reordering (0x8000)
    and as the default variant chooses (the tuner times both orders), timed alike; all
    must be bit-identical."""
    from vct import scenes
    from vct.camera import Camera
    w, h = args.width, args.height
    ao, nm = ctx.download_voxels()
    gb = tuple(torch.from_numpy(a).to(dev) for a in scenes.gbuffer_rand(ao, nm, ctx.aabb_min, ctx.extent, w, h,
                                                                         seed=42))
    del ao, nm
    eye = [float(x) for x in Camera().position]
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    outs, ms, form = {}, {}, {}
    reps = max(3, args.steps // 4)
    auto = args.variant & ~0x4008000
    for v in (auto | 0x4000000, auto | 0x8000, auto):   # screen order forced / reordering forced / tuner's choice
        d = torch.empty((h, w, 4), device=dev)
        sp = torch.empty((h, w, 4), device=dev)
        if v & 0x4000000:      # the counting pass, once (screen order)
            ctx.trace_device(*gb, w, h, eye, d, sp, cone_steps=cnt, variant=v)
            counted = (d.clone(), sp.clone())
        # a forced order holds at once; the default variant may first re-time the choice it made
        # on G_scene under the same workload key (drift watch), so it settles longer
        form[v] = settle_form(ctx, torch, lambda: ctx.trace_device(*gb, w, h, eye, d, sp, variant=v),
                              stable=6 if v != auto else 24)
        ctx.trace_device(*gb, w, h, eye, d, sp, variant=v)     # warm
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        e[0].record(stream)
        for _ in range(reps):
            ctx.trace_device(*gb, w, h, eye, d, sp, variant=v)
        e[1].record(stream)
        torch.cuda.synchronize()
        ms[v] = e[0].elapsed_time(e[1]) / reps
        outs[v] = (d, sp)
    steps = int(cnt[0].item())
    (a0, a1), (b0, b1), (c0, c1) = outs.values()
    t0, t1, t2 = ms.values()
    loop = frame_loop(torch, ctx, gb, w, h, eye, stream, args.frame_loop, variant=auto) if args.frame_loop else None
    key = profile_key(args.n, w, h, args.scene, "rand", args.n_diffuse, not args.no_spec, args.variant, 1)
    rec, reason = load_profile(args.profile_json, key)
    # whole frames are timed here (the reorder keys and sort included), so the roofline's
    # live time is the record's own rocprofv3 K4 duration
    roof = roofline(rec, reason, None, None, w * h, args.profile_json, key, steps=steps)
    return {"gbuffer": "G_rand (seed 42), same grid", "frame_cone_steps": steps, "frames": reps, "_loop": loop,
            "roofline": roof,
            "screen_order_ms": round(t0, 4), "reordered_ms": round(t1, 4), "default_ms": round(t2, 4),
            "screen_order_Mcone_steps_s": round(steps / t0 / 1e3, 2),
            "reordered_Mcone_steps_s": round(steps / t1 / 1e3, 2),
            "default_Mcone_steps_s": round(steps / t2 / 1e3, 2),
            "speedup": round(t0 / t1, 3), "k4_forms": list(form.values()),
            "default_choice": "ray reordering" if form[auto] >= 0 and form[auto] & 2 else "screen order",
            "bitexact": bool(torch.equal(a0, b0) and torch.equal(a1, b1) and torch.equal(a0, c0) and
                             torch.equal(a1, c1)),
            "timed_equals_counting": bool(all(torch.equal(x, counted[0]) and torch.equal(y, counted[1])
                                              for x, y in outs.values()))}


def run(args, world):
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; VCT_DIST_BACKEND=gloo rehearses the N>1 path with
    # several ranks on one device (RCCL refuses two ranks per GPU)
    backend = os.environ.get("VCT_DIST_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    dev_index = local_rank % ndev if backend != "nccl" else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        # a collective that cannot complete (a rank died or hangs) ends every rank with an
        # error after 120 s -- inside the driver's 600 s bench limit -- instead of torch's
        # default 10-minute timeout killing the run without a line
        pg_timeout = datetime.timedelta(seconds=float(os.environ.get("VCT_PG_TIMEOUT_S", "120")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout)
        else:
            dist.init_process_group(backend, timeout=pg_timeout)

    from vct import Context, scenes

    n, w, h = args.n, args.width, args.height
    spec = not args.no_spec
    g0, E = scenes.grid_for_unit_box(n)
    ctx = Context(n, g0, E, aniso=True, n_diffuse=args.n_diffuse, specular=spec, device=dev_index)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)

    progress(rank, f"metric workload: {args.scene} {n}^3 {w}x{h}, {world} rank(s)")
    m = measure_scene(args, torch, dist, ctx, args.scene, rank, world, dev, stream, relight_roofs=rank == 0)
    progress(rank, f"metric done: {m['value']:.0f} Mcone-steps/s")
    key = profile_key(n, w, h, args.scene, args.gbuffer, args.n_diffuse, spec, args.variant, world)
    rec, reason = load_profile(args.profile_json, key)
    roof = roofline(rec, reason, m["k4_kernel_ms_avg"], m["local_texels"], m["local_valid"], args.profile_json, key,
                    steps=m["local_steps"])
    if roof.get("frac") is not None and m["ms_per_step"] > 0:
        # the same per-launch work over the pipelined frame time: with frame overlap a launch's
        # own start-to-end time includes the other frame's share of the chip, so the rate the
        # timed loop sustains is work per frame / ms per step
        r_ = roof["frac"] * m["k4_kernel_ms_avg"] / m["ms_per_step"]
        roof["pipelined"] = {"achieved": round(roof["achieved"] * m["k4_kernel_ms_avg"] / m["ms_per_step"], 1),
                             "frac": round(r_, 4), "ms_per_frame": round(m["ms_per_step"], 4),
                             "basis": "per-launch counts / (timed wall time / K)"}

    result = None
    if rank == 0:
        result = {
            "metric": METRIC,
            "value": round(m["value"], 2),
            "unit": "Mcone-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(m["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: procedural '{args.scene}' scene{STAND_IN.get(args.scene, '')}, G_{args.gbuffer} G-buffer",
            "config": {
                "workload": f"cone trace K4, {n}^3 aniso RGBA32F grid, {w}x{h}, "
                            f"{args.n_diffuse} diffuse + {1 if spec else 0} specular cones",
                "grid": n, "width": w, "height": h, "scene": args.scene, "gbuffer": args.gbuffer,
                "n_diffuse": args.n_diffuse, "specular": spec, "parallelism": f"screen-tiles x{world}",
                "exchange": args.exchange if world > 1 else None, "variant": args.variant,
            },
        }
        for k_ in ("frame_cone_steps", "valid_px"):
            result[k_] = m[k_]
        # latency beside throughput: `value` pipelines consecutive frames (frame f+1's trace
        # fills the tail of frame f's launch), so a launch inside the loop runs longer from
        # start to end than alone; a renderer that presents each frame before tracing the
        # next gets `value_single_launch` (frame steps / the launch alone)
        if world == 1:
            result["value_single_launch"] = round(m["frame_cone_steps"] / m["k4_kernel_ms_avg"] / 1e3, 2)
        else:
            tr, ex = m.get("trace_ms_max_rank"), m.get("gather_ms" if args.exchange == "present" else "allgather_ms")
            result["value_unpipelined"] = round(m["frame_cone_steps"] / (tr + ex) / 1e3, 2) if tr and ex else None
        result["latency"] = {"k4_launch_ms_alone": round(m["k4_kernel_ms_avg"], 4),
                             "k4_launch_ms_alone_min_max": [round(m["k4_kernel_ms_min"], 4), round(m["k4_kernel_ms_max"], 4)],
                             "k4_launch_ms_in_pipelined_loop": round(m["k4_kernel_ms_avg_overlapped"], 4),
                             "frame_ms_pipelined": round(m["ms_per_step"], 4),
                             "frames_in_flight": 2 if m["overlap"] or world > 1 else 1}
        result["k4_kernel_ms_avg"] = round(m["k4_kernel_ms_avg"], 4)
        result["k4_kernel_ms_median"] = round(m["k4_kernel_ms_median"], 4)
        result["k4_kernel_ms_avg_overlapped"] = round(m["k4_kernel_ms_avg_overlapped"], 4)
        result["frame_overlap"] = "two trace streams" if m["overlap"] else "one stream"
        result["overlap_tune"] = m["overlap_tune"]
        result["k4_form"] = form_name(m["k4_form"])
        result["k4_form_alone"] = form_name(m["k4_form_alone"])
        result["timed_equals_counting"] = m["timed_equals_counting"]
        # (the timed loops here overlap frames or follow overlapped ones: blockIdx order)
        result["k4_dispatch"] = ("blockIdx order through the XCD map; each XCD's units longest first (from the "
                                 "previous launch's per-unit wave durations) only in launches of <= 4 generations of "
                                 "waves that do not overlap another frame (DESIGN 13.5)")
        for k_ in ("k1_voxelize_ms", "k2_inject_ms", "k3_mips_ms", "k3_mips_relight_ms", "grid_bcast_ms", "frame_relight_ms",
                   "frame_relight_bcast_ms", "frame_relight_replicated_ms", "replicated_k2_equals_bcast",
                   "trace_ms_max_rank", "gather_ms", "allgather_ms", "k1_roofline", "k2_roofline", "k3_roofline"):
            if k_ in m:
                result[k_] = m[k_]
        result["roofline"] = roof
        result["cpu_baseline"] = None
        result["frame_loop"] = None
        if world == 1 and not args.no_cpu_baseline:
            host = tuple(t_.cpu().numpy() for t_ in m["_gb"])
            result["cpu_baseline"] = cpu_baseline(ctx, n, g0, E, host, m["_eye"], args.n_diffuse, spec,
                                                  m["_steps_px"].cpu().numpy().astype(np.uint32), args.cpu_seconds)
    if world == 1 and args.frame_loop:
        loop_scene = frame_loop(torch, ctx, m["_gb"], w, h, m["_eye"], stream, args.frame_loop, variant=args.variant)
        result["frame_loop"] = {f"G_{args.gbuffer}": loop_scene}
        progress(rank, "frame loop done")
    capi = None
    if world > 1:
        if os.environ.get("VCT_DIST_BACKEND", "nccl") == "nccl":
            # a failure on any rank (the C-ABI returns VCT_ECOMM after its deadline and aborts
            # its communicator) is recorded, agreed on over the torch group, and the line goes on
            err = None
            try:
                capi = capi_leg(args, torch, dist, ctx, rank, world, dev, stream, m["_gb"], m["_eye"])
            except Exception as e:   # noqa: BLE001 -- reported in the JSON line
                err = f"{type(e).__name__}: {e}"[:300]
                capi = None
            if max_over_ranks(torch, dist, dev, [0.0 if err is None else 1.0], world)[0] != 0.0:
                capi = {"error": err or "failed on another rank", "present_equal": None, "allgather_equal": None,
                        "bcast_equal": None}
        else:
            capi = {"note": "skipped: the C-ABI RCCL path needs one GPU per rank (VCT_DIST_BACKEND is not nccl)",
                    "present_equal": None, "allgather_equal": None, "bcast_equal": None,
                    "present_frame_ms": None, "allgather_frame_ms": None, "bcast_ms": None}
        if rank == 0:
            result["capi"] = capi
            # what the collectives ran over: torch's process group and the C-ABI's own
            # RCCL communicator (vct_comm_rank after vct_comm_init)
            result["rccl"] = {"backend": dist.get_backend(), "pg_world": dist.get_world_size(),
                              "pg_timeout_s": float(os.environ.get("VCT_PG_TIMEOUT_S", "120")),
                              "vct_comm_nranks": (capi or {}).get("vct_comm_nranks"),
                              "vct_comm_ranks_match": (capi or {}).get("vct_comm_ranks_match")}
    del m
    torch.cuda.empty_cache()
    st = (args.stress or "").strip()
    if st == "rand" and world == 1 and args.gbuffer == "scene":
        progress(rank, "stress (G_rand)")
        result["stress"] = stress_rand(args, torch, ctx, dev, stream)
        loop = result["stress"].pop("_loop")
        if loop is not None:
            result["frame_loop"]["G_rand"] = loop
        torch.cuda.empty_cache()
    sec = (args.secondary or "").strip()
    if sec and sec != "none" and sec != args.scene:
        # the same size on a non-flat scene (varied normals: fewer combined-face bricks)
        progress(rank, f"secondary: {sec}")
        s2 = measure_scene(args, torch, dist, ctx, sec, rank, world, dev, stream)
        if rank == 0:
            result["secondary"] = {
                "scene": sec + STAND_IN.get(sec, ""), "value": round(s2["value"], 2), "unit": "Mcone-steps/s",
                "ms_per_step": round(s2["ms_per_step"], 4), "k4_kernel_ms_avg": round(s2["k4_kernel_ms_avg"], 4),
                "frame_cone_steps": s2["frame_cone_steps"], "valid_px": s2["valid_px"],
                "k1_voxelize_ms": s2["k1_voxelize_ms"], "k4_form": form_name(s2["k4_form"]),
                "timed_equals_counting": s2["timed_equals_counting"],
                "value_single_launch": round(s2["frame_cone_steps"] / s2["k4_kernel_ms_avg"] / 1e3, 2)
                if world == 1 else None,
            }
            key2 = profile_key(n, w, h, sec, args.gbuffer, args.n_diffuse, spec, args.variant, world)
            result["secondary"]["roofline"] = roofline(*load_profile(args.profile_json, key2), s2["k4_kernel_ms_avg"],
                                                       s2["local_texels"], s2["local_valid"], args.profile_json, key2,
                                                       steps=s2["local_steps"])
            if "trace_ms_max_rank" in s2:
                result["secondary"]["trace_ms_max_rank"] = s2["trace_ms_max_rank"]
        del s2
    ctx.close()
    torch.cuda.empty_cache()
    mc = [c.strip() for c in (args.multi_config or "").split(",") if c.strip() and c.strip() != "none"]
    if mc:
        out = {}
        for name in mc:
            cfg = MULTI_CONFIGS[name]
            if cfg["ranks"] is not None and world not in cfg["ranks"]:
                continue
            progress(rank, f"multi_config {name}")
            out[name] = measure_config(args, torch, dist, rank, world, dev, stream, cfg)
        if rank == 0:
            result["multi_config"] = out
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        emit(result)


if __name__ == "__main__":
    main()
