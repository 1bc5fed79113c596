#!/bin/bash
# The round's final GPU evidence on one box: the default bench line (with the CPU
# baseline), a rocprofv3 kernel trace + stats of the same command (profiles/), smoke().
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
timeout -k 10 500 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
rc=$?; echo "bench rc=$rc"; head -c 300 gpurun_out/bench_final.json; echo
[ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/trace.stdout 2> $OUT/trace.stderr
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/trace.stderr; exit $rc; }
# keep the summaries (the full per-dispatch trace of a whole bench run exceeds what gpurun copies back)
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/ \;
python3 - $OUT <<'PY'
import csv, glob, json, re, sys
out = sys.argv[1]
f = glob.glob(out + "/trace/**/*kernel_trace.csv", recursive=True)[0]
d = {}
for r in csv.DictReader(open(f)):
    if re.search(r"k4_trace<[^>]*, false(?:, \d+)?>\(", r["Kernel_Name"]):   # the counter-free (timed) form
        d.setdefault(r["Kernel_Name"] + " grid " + r["Grid_Size_X"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
json.dump({k: {"dispatches": len(v), "avg_ms": sum(v) / len(v) / 1e6} for k, v in d.items()}, open(out + "/k4_timed_dispatches.json", "w"), indent=1)
PY
rm -rf $OUT/trace
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
exit $rc
