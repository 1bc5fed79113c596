#!/bin/bash
# rocprofv3 records of every line bench.py reports (one GPU; the roofline inputs):
# for each workload (tools/pmc_workload.py: c3 = the metric, courtyard = `secondary`,
# rand = `stress`, c4 / c5 = `multi_config`; "wl:N" = rank 0's launch of the N-rank
# split) two rocprofv3 runs of the same command, each with --kernel-trace and one
# counter group (the per-block slot limits of MI355X_MICROARCH.md 'rocprofv3 PMC
# slots': 8 SQ + TCC hit / miss + WRITE_SIZE; FETCH_SIZE + the L2's atomic requests + the
# GPU-busy clock count GRBM_GUI_ACTIVE, summed over the 8 XCDs: the effective clock),
# then tools/make_pmc_records.py writes the records, stamped with the library's sha256.
#   TAG=r4a WLS="c3 courtyard rand c4 c5 c3:2 c3:4 c3:8" bash tools/pmc_all.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r4}
WLS=${WLS:-"c3 courtyard rand c4 c5 c3:2 c3:4 c3:8 courtyard:2 courtyard:4 courtyard:8 c4:2 c4:4 c4:8 c5:8"}
ROOT=gpurun_out/pmc_$TAG
mkdir -p $ROOT
faulted() { grep -qE "HSA_STATUS_ERROR|Memory access fault|APERTURE_VIOLATION|GPU core dump" "$@"; }
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for spec in $WLS; do
  wl=${spec%%:*}; N=1
  [ "$spec" != "$wl" ] && N=${spec##*:}
  OUT=$ROOT/${wl}_ranks$N
  mkdir -p $OUT
  for pass in a b; do
    if [ $pass = a ]; then PMC="$SQ TCC_HIT_sum TCC_MISS_sum WRITE_SIZE"; else PMC="FETCH_SIZE TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE"; fi
    timeout -s KILL ${PASS_TIMEOUT:-240} rocprofv3 --kernel-trace --pmc $PMC -d $OUT/$pass -o $pass --output-format csv \
        -- python3 tools/pmc_workload.py --wl $wl --world $N --rank 0 > $OUT/$pass.stdout 2> $OUT/$pass.stderr
    rc=$?
    echo "$spec pass $pass rc=$rc $(tail -c 300 $OUT/$pass.stdout)"
    if faulted $OUT/$pass.stderr; then echo "FAULT in $spec $pass"; exit 99; fi
    if [ $rc -ne 0 ]; then tail -20 $OUT/$pass.stderr; exit $rc; fi
  done
done
python3 tools/make_pmc_records.py $ROOT --tag $TAG > $ROOT/records.txt && cat $ROOT/records.txt
