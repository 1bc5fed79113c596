#!/bin/bash
# rocprofv3 passes over a short bench run (kernel trace + stats, then separate
# PMC passes).  Output under gpurun_out/prof_<tag>/.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
faulted() { grep -qE "HSA_STATUS_ERROR|Memory access fault|APERTURE_VIOLATION" "$@"; }
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $BARGS \
      > $OUT/$name.stdout 2> $OUT/$name.stderr
  local rc=$?
  echo "$name rc=$rc"
  if faulted $OUT/$name.stderr; then echo "FAULT in $name"; exit 99; fi
  if [ $rc -ne 0 ]; then tail -20 $OUT/$name.stderr; exit $rc; fi
}
run trace --kernel-trace --stats
if [ -n "$LIST" ]; then timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true; fi
if [ -n "$PMC_SETS" ]; then IFS=';' read -ra SETS <<< "$PMC_SETS"
else SETS=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"); fi
for p in "${SETS[@]}"; do
  n=pmc_$(echo $p | tr ' ' '_' | cut -c1-40)
  run $n --pmc $p
done
find $OUT -name "*.csv" | head -50
