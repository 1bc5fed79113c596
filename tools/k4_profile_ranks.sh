#!/bin/bash
# Per-rank rocprofv3 records for bench.py's roofline at N > 1 (one GPU): for each
# world size N, rank 0's own K4 launch of the N-rank screen-tile split
# (tools/rank_emul.py --pmc-world N) under a kernel-trace + stats pass and one PMC
# pass per counter group, then tools/make_k4_profile.py with WORLD_SIZE=N writes
# the `... ranksN` record stamped with the library's sha256.
#   TAG=r3x WORLDS="2 4 8" bash tools/k4_profile_ranks.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r3}
WORLDS=${WORLDS:-"2 4 8"}
faulted() { grep -qE "HSA_STATUS_ERROR|Memory access fault|APERTURE_VIOLATION|GPU core dump" "$@"; }
for N in $WORLDS; do
  OUT=gpurun_out/prof_${TAG}_ranks$N
  mkdir -p $OUT
  run() {  # name, rocprof args...
    local name=$1; shift
    timeout -s KILL ${PASS_TIMEOUT:-180} rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- \
        python3 tools/rank_emul.py --pmc-world $N --pmc-rank 0 > $OUT/$name.stdout 2> $OUT/$name.stderr
    local rc=$?
    echo "ranks$N $name rc=$rc"
    if faulted $OUT/$name.stderr; then echo "FAULT in $name"; exit 99; fi
    if [ $rc -ne 0 ]; then tail -20 $OUT/$name.stderr; exit $rc; fi
  }
  run trace --kernel-trace --stats
  run pmc_fetch --pmc FETCH_SIZE
  run pmc_write --pmc WRITE_SIZE
  run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
  run pmc_tcc --pmc TCC_HIT_sum TCC_MISS_sum
  WORLD_SIZE=$N python3 tools/make_k4_profile.py $OUT --tag ${TAG}_ranks$N --steps 10 > $OUT/record.json || exit 1
  echo "ranks$N record: $(python3 -c "import json;d=json.load(open('$OUT/record.json'));k=list(d)[0];print(k, d[k]['duration_ms'], d[k]['SQ_INSTS_SALU'])")"
done
