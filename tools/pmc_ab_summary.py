#!/usr/bin/env python3
"""Mean per-dispatch PMC values of the K4 kernels in a tools/pmc_ab.sh run.

    python tools/pmc_ab_summary.py gpurun_out/pmc_ab_<tag>
"""
import collections
import csv
import glob
import sys


def main():
    root = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        names = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k4_trace" not in r["Kernel_Name"]:
                    continue
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in per.items():
            acc[names[d][:80]][c].append(v)
    for k, cs in acc.items():
        print(k)
        for c, vs in sorted(cs.items()):
            print(f"  {c:28s} {sum(vs) / len(vs):16.4g}  (n={len(vs)})")


if __name__ == "__main__":
    main()
