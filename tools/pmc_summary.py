#!/usr/bin/env python3
"""Summarise rocprofv3 PMC / kernel-trace CSVs per kernel (mean per dispatch).

usage: pmc_summary.py <prof_dir> [kernel_substring]
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 units); on gfx950
FETCH_SIZE under-counts wide streaming reads by 2x (MI355X_MICROARCH.md
'HBM'), so `hbm_read_bytes_corrected` doubles it.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "k4_trace"
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if key in r["Kernel_Name"]:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if key in r["Kernel_Name"]:
                    durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    if durs:
        out["duration_ns_mean"] = sum(durs) / len(durs)
        out["dispatches"] = len(durs)
    if "FETCH_SIZE" in out:
        out["hbm_read_bytes_corrected"] = out["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in out:
        out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in out and "TCC_MISS_sum" in out:
        out["l2_hit_rate"] = out["TCC_HIT_sum"] / max(1.0, out["TCC_HIT_sum"] + out["TCC_MISS_sum"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
