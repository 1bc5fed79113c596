#!/bin/bash
# Memory-pipeline PMC of the timed K4 form (texture address / data units, vector L1):
# one rocprofv3 --pmc pass per counter group (per-block slot limits, MI355X_MICROARCH.md),
# over the same short bench command; per-pass summaries in gpurun_out/pmc_mem_<tag>/.
#   TAG=x LIB=vct/libvct_hip_foo.so bash tools/pmc_mem.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-mem}
OUT=gpurun_out/pmc_mem_$TAG
mkdir -p $OUT
[ -n "$LIB" ] && export VCT_LIB=$PWD/voxel-based-global-illumination_amd/$LIB
KEY=${KEY:-"k4_trace<true, 5, false, true, 2, true, false, true, false>"}   # the occupancy form (atrium)
BARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline --secondary none --stress none"}
i=0
for P in ${PASSES:-"GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_BUSY_avr" "TD_TD_BUSY_sum TD_BUSY_avr" \
    "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
    "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
    "SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CU_CYCLES"}; do
  i=$((i+1))
  timeout -s KILL ${PASS_TIMEOUT:-60} rocprofv3 --pmc $P -d $OUT/p$i -o p --output-format csv -- python3 bench.py $BARGS \
      > $OUT/p$i.stdout 2> $OUT/p$i.stderr
  rc=$?
  echo "pass $i ($P) rc=$rc"
  if grep -qE "HSA_STATUS_ERROR|Memory access fault|APERTURE_VIOLATION|GPU core dump" $OUT/p$i.stderr; then echo FAULT; exit 99; fi
  if [ $rc -ne 0 ]; then tail -3 $OUT/p$i.stderr; [ $rc -ge 124 ] && exit $rc; continue; fi
  python3 tools/pmc_summary.py $OUT/p$i "$KEY" > $OUT/p$i.json && cat $OUT/p$i.json
done
