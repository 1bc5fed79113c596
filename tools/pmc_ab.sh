#!/bin/bash
# PMC counters of tools/ab.py variants (one counter set per rocprofv3 pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ab_${TAG:-x}
mkdir -p $OUT
VARS=${VARS:-3,0}
IFS=';' read -ra SETS <<< "${PMC_SETS:-SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH}"
i=0
for p in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $p -d $OUT/p$i -o p$i --output-format csv -- python3 tools/ab.py --variants $VARS --rounds 1 --reps 2 > $OUT/p$i.out 2> $OUT/p$i.err
  rc=$?; echo "pass $i rc=$rc"
  if grep -qE "HSA_STATUS_ERROR|Memory access fault" $OUT/p$i.err; then echo FAULT; exit 99; fi
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.err; exit $rc; fi
done
