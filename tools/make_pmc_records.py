#!/usr/bin/env python3
"""Roofline records from tools/pmc_all.sh's rocprofv3 runs (the inputs of bench.py's
per-line `roofline` and of its `k1_roofline` / `k2_roofline` / `k3_roofline`).

    make_pmc_records.py <pmc_root> --tag T [--merge]

For every workload directory <pmc_root>/<wl>_ranks<N>/{a,b} (two rocprofv3 runs of
tools/pmc_workload.py, each with --kernel-trace and one counter group):
  * K4: the timed form's (the k4_trace instantiation without counters) most frequent
    (kernel, grid) -- the form the tuner settled on -- averaged per dispatch; the
    duration from pass a's kernel trace; HBM = (2 FETCH_SIZE + WRITE_SIZE) x 1024 per
    launch (gfx950: FETCH_SIZE counts half the bytes of wide reads, MI355X_MICROARCH.md
    'HBM');
  * K1 / K2 / K3 (one-rank workloads): every kernel the voxelize / inject / build_mips
    calls launch, per call: sum over that call's kernels of the per-dispatch means x
    the dispatches per call, and the summed kernel durations.
Records carry the sha256 of the libvct_hip.so they were measured on (bench.py uses a
record only for that build).  --merge writes them into profiles/k4_counters.json
(keyed like bench.profile_key) and profiles/relight_counters.json (keyed
"<n>^3 <scene>").
"""
import argparse
import csv
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
TIMED = re.compile(r"k4_trace<[^>]*, false(?:, \d+)?>\(")   # the counter-free form (any waves per workgroup)
# kernels of each relight call (vct_voxelize.hip, vct_mips.hip); k2_list builds K1's occupied list
STAGES = {
    # K1's scans are the 64-bit ones (vct_reorder.hip's counting sort has k_scan_* of 32 bits)
    "k1": re.compile(r"^(?:void )?(?:vct::\(anonymous namespace\)::)?(k1_\w+|k_scan_\w+(?=\(unsigned long long)|k2_list)\b"),
    "k2": re.compile(r"^(?:void )?(?:vct::\(anonymous namespace\)::)?(k2_(?:coarse|shade|walk|inject)\w*)"),
    "k3": re.compile(r"^(?:void )?(?:vct::\(anonymous namespace\)::)?(k3_\w+)"),
}


def rows(d, pat):
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def stage_of(name):
    for st, rx in STAGES.items():
        m = rx.search(name)
        if m:
            return st, m.group(1)
    return None, None


def load(wdir):
    """-> (driver JSON, {pass: {dispatch_id: {kernel, grid, dur_ns, counters}}})"""
    info, passes = None, {}
    for p in ("a", "b"):
        out = os.path.join(wdir, f"{p}.stdout")
        if info is None and os.path.exists(out):
            for line in open(out):
                line = line.strip()
                if line.startswith("{"):
                    info = json.loads(line)
        disp = {}
        for r in rows(os.path.join(wdir, p), "*kernel_trace.csv"):
            disp[int(r["Dispatch_Id"])] = {"kernel": r["Kernel_Name"], "grid": int(r["Grid_Size_X"]),
                                           "dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "ctr": {}}
        for r in rows(os.path.join(wdir, p), "*counter_collection.csv"):
            did = int(r["Dispatch_Id"])
            e = disp.setdefault(did, {"kernel": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "dur_ns": None,
                                      "ctr": {}})
            e["ctr"][r["Counter_Name"]] = e["ctr"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        passes[p] = disp
    return info, passes


def k4_record(passes):
    a = passes["a"]
    groups = {}
    for did, e in a.items():
        if TIMED.search(e["kernel"]):
            groups.setdefault((e["kernel"], e["grid"]), []).append(did)
    if not groups:
        return None
    key = max(groups, key=lambda k: len(groups[k]))
    rec = {"kernel": key[0], "grid_threads": key[1], "dispatches": len(groups[key])}
    durs = [a[d]["dur_ns"] for d in groups[key] if a[d]["dur_ns"] is not None]
    rec["duration_ms"] = sum(durs) / len(durs) / 1e6 if durs else None
    for p, disp in passes.items():
        sel = [e for e in disp.values() if (e["kernel"], e["grid"]) == key and e["ctr"]]
        names = set(c for e in sel for c in e["ctr"])
        for c in sorted(names):
            v = [e["ctr"][c] for e in sel if c in e["ctr"]]
            rec[c] = sum(v) / len(v)
        # effective shader clock of the same dispatches: GRBM_GUI_ACTIVE counts busy cycles
        # summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back); read high below ~0.3 ms
        ck = [e["ctr"]["GRBM_GUI_ACTIVE"] / 8.0 / e["dur_ns"] for e in sel
              if "GRBM_GUI_ACTIVE" in e["ctr"] and e["dur_ns"]]
        if ck:
            rec["effective_clock_ghz"] = sum(ck) / len(ck)
    return rec


def first_build(disp, st):
    """dispatch ids of stage st's first call: the earliest dispatch of each (kernel, grid)"""
    first = {}
    for did in sorted(disp):
        e = disp[did]
        s, _ = stage_of(e["kernel"])
        if s == st:
            first.setdefault((e["kernel"], e["grid"]), did)
    return set(first.values())


def stage_records(passes, calls, drop_first=()):
    """per relight stage: counters and kernel time per call, and the per-kernel split.
    Stages in drop_first lose their first call (e.g. K3's full build before the relight
    builds the workload measures; calls[st] counts the calls kept)."""
    out = {}
    for st in STAGES:
        per_kernel = {}
        for p, disp in passes.items():
            skip = first_build(disp, st) if st in drop_first else set()
            for did, e in disp.items():
                if did in skip:
                    continue
                s, kname = stage_of(e["kernel"])
                if s != st:
                    continue
                pk = per_kernel.setdefault(kname, {"dispatches": {}, "dur": [], "ctr": {}})
                pk["dispatches"][p] = pk["dispatches"].get(p, 0) + 1
                if p == "a" and e["dur_ns"] is not None:
                    pk["dur"].append(e["dur_ns"])
                for c, v in e["ctr"].items():
                    pk["ctr"][c] = pk["ctr"].get(c, 0.0) + v
        if not per_kernel:
            continue
        n = calls[st]
        tot = {"calls": n, "kernels": {}}
        sums, ms = {}, 0.0
        for kname, pk in sorted(per_kernel.items()):
            kms = sum(pk["dur"]) / 1e6 / n
            ms += kms
            tot["kernels"][kname] = {"ms_per_call": round(kms, 5), "dispatches_per_call": pk["dispatches"].get("a", 0) / n}
            for c, v in pk["ctr"].items():
                sums[c] = sums.get(c, 0.0) + v / n
        tot["kernel_ms_per_call"] = ms
        tot.update({c: v for c, v in sorted(sums.items())})
        out[st] = tot
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--merge", action="store_true")
    a = ap.parse_args()
    import bench
    sha = bench.lib_sha256()
    k4, rel = {}, {}
    for wdir in sorted(glob.glob(os.path.join(a.root, "*_ranks*"))):
        info, passes = load(wdir)
        if info is None or "a" not in passes:
            print(f"{wdir}: incomplete", file=sys.stderr)
            continue
        rec = k4_record(passes)
        if rec is None:
            continue
        rec.update({"lib_sha256": sha, "tag": a.tag, "source": os.path.relpath(wdir, REPO),
                    "cone_steps": info["cone_steps"], "texel_fetches": info["texel_fetches"],
                    "valid_px": info["valid_px"], "form": info["form_name"],
                    "correction": "hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halves wide reads)"})
        if "FETCH_SIZE" in rec and "WRITE_SIZE" in rec:
            rec["hbm_bytes_per_launch"] = int(2 * rec["FETCH_SIZE"] * 1024 + rec["WRITE_SIZE"] * 1024)
        if "TCC_HIT_sum" in rec:
            rec["l2_hit_rate"] = rec["TCC_HIT_sum"] / max(1.0, rec["TCC_HIT_sum"] + rec["TCC_MISS_sum"])
        if rec.get("SQ_WAVE_CYCLES"):
            rec["issue_active"] = rec["SQ_ACTIVE_INST_ANY"] / rec["SQ_WAVE_CYCLES"]
        rec["valu_per_cone_step"] = rec.get("SQ_INSTS_VALU", 0) / max(1, info["cone_steps"])
        rec["salu_per_cone_step"] = rec.get("SQ_INSTS_SALU", 0) / max(1, info["cone_steps"])
        k4[info["key"]] = rec
        print(f"{info['key']}: {rec['duration_ms']:.4f} ms, VALU/step {rec['valu_per_cone_step']:.3f}, "
              f"SALU/step {rec['salu_per_cone_step']:.3f}, issue {rec.get('issue_active', 0):.3f}, "
              f"form {info['form_name']}")
        if info["world"] == 1:
            n_, scene = info["key"].split(" ")[0], info["key"].split(" ")[2]
            # K3: the first build after K1 is full, the later ones are relight builds (only
            # the blocks with an occupied voxel, no K4 maps): the record is of those
            full1 = bool(info.get("k3_first_build_full"))
            st = stage_records(passes, {"k1": info["k1_calls"], "k2": info["relight_calls"],
                                        "k3": info["relight_calls"] - (1 if full1 else 0)},
                               drop_first=("k3",) if full1 else ())
            if full1 and "k3" in st:
                st["k3"]["build"] = "relight (first full build after K1 dropped)"
            for s_, v in st.items():
                v.update({"lib_sha256": sha, "tag": a.tag, "source": os.path.relpath(wdir, REPO)})
                if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
                    v["hbm_bytes_per_call"] = int(2 * v["FETCH_SIZE"] * 1024 + v["WRITE_SIZE"] * 1024)
                if "TCC_HIT_sum" in v:
                    v["l2_hit_rate"] = v["TCC_HIT_sum"] / max(1.0, v["TCC_HIT_sum"] + v["TCC_MISS_sum"])
                if "TCC_EA0_ATOMIC_sum" in v:
                    v["atomic_bytes_per_call"] = int(v["TCC_EA0_ATOMIC_sum"] * 64)
                if v.get("SQ_WAVE_CYCLES"):
                    v["issue_active"] = v["SQ_ACTIVE_INST_ANY"] / v["SQ_WAVE_CYCLES"]
                    v["wait_any"] = v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"]
                rel.setdefault(f"{n_} {scene}", {})[s_] = v
                split = ", ".join("%s=%.4f" % (k_, x["ms_per_call"]) for k_, x in v["kernels"].items())
                print(f"  {n_} {scene} {s_}: {v['kernel_ms_per_call']:.4f} ms/call, {split}")
    out = os.path.join(REPO, "gpurun_out", f"pmc_records_{a.tag}.json")
    with open(out, "w") as fh:
        json.dump({"k4": k4, "relight": rel}, fh, indent=1, sort_keys=True)
    if a.merge:
        for name, new in (("k4_counters.json", k4), ("relight_counters.json", rel)):
            path = os.path.join(REPO, "profiles", name)
            db = json.load(open(path)) if os.path.exists(path) else {}
            db.update(new)
            with open(path, "w") as fh:
                json.dump(db, fh, indent=1, sort_keys=True)
            print(f"{path}: {len(db)} entries")


if __name__ == "__main__":
    main()
