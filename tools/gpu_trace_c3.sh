#!/bin/bash
# rocprofv3 kernel trace + stats of the metric workload alone with frame overlap off, so
# every timed K4 launch runs by itself: its average must agree with the bench line's
# k4_kernel_ms_avg (profiles/<round>_<tag>_c3_*)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r4}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py --steps 50 --overlap off --no-cpu-baseline --secondary none --stress none --multi-config none --frame-loop 0 > $OUT/c3.json 2> $OUT/c3.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/c3.err; exit $rc; }
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/c3_kernel_stats.csv \;
python3 - $OUT <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
f = glob.glob(out + "/trace/**/*kernel_trace.csv", recursive=True)[0]
d = {}
for r in csv.DictReader(open(f)):
    if "k4_trace" in r["Kernel_Name"]:
        d.setdefault(r["Kernel_Name"] + " grid " + r["Grid_Size_X"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
line = json.loads(open(out + "/c3.json").read())
json.dump({"bench_k4_kernel_ms_avg": line["k4_kernel_ms_avg"], "bench_ms_per_step": line["ms_per_step"],
           "dispatches": {k: {"n": len(v), "avg_ms": sum(v) / len(v) / 1e6, "min_ms": min(v) / 1e6} for k, v in d.items()}},
          open(out + "/c3_k4_dispatches.json", "w"), indent=1)
print(open(out + "/c3_k4_dispatches.json").read())
PY
rm -rf $OUT/trace
