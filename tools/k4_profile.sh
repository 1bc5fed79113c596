#!/bin/bash
# rocprofv3 evidence for bench.py's roofline (one GPU): a kernel-trace + stats pass,
# then one PMC pass per counter group (separate runs, MI355X_MICROARCH.md 'rocprofv3
# PMC slots'), all over the same short bench command; then
# tools/make_k4_profile.py writes the timed K4 form's per-launch record, keyed by
# workload and stamped with the library's sha256, to gpurun_out/k4_counters_<tag>.json
# (merge it into profiles/k4_counters.json with tools/make_k4_profile.py --merge).
#   TAG=r2a BENCH_ARGS="..." bash tools/k4_profile.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline --secondary none --stress none"}
faulted() { grep -qE "HSA_STATUS_ERROR|Memory access fault|APERTURE_VIOLATION|GPU core dump" "$@"; }
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -s KILL ${PASS_TIMEOUT:-240} rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $BARGS \
      > $OUT/$name.stdout 2> $OUT/$name.stderr
  local rc=$?
  echo "$name rc=$rc"
  if faulted $OUT/$name.stderr; then echo "FAULT in $name"; exit 99; fi
  if [ $rc -ne 0 ]; then tail -20 $OUT/$name.stderr; exit $rc; fi
}
run trace --kernel-trace --stats
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run pmc_tcc --pmc TCC_HIT_sum TCC_MISS_sum
python3 tools/make_k4_profile.py $OUT --tag $TAG $BARGS > $OUT/record.json && cat $OUT/record.json
