#!/bin/bash
# One rocprofv3 --pmc pass per library over the same short bench command (K4 only):
#   PMC="SQ_WAVES SQ_INSTS_VALU" bash tools/pmc_libs.sh tag lib1.so lib2.so ...
# -> gpurun_out/pmc_<tag>_<i>/  (summarised by tools/pmc_ab_summary.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; shift
i=0
for L in "$@"; do
  i=$((i+1))
  out=gpurun_out/pmc_${tag}_$i
  mkdir -p $out
  echo "$L" > $out/lib.txt
  VCT_LIB=$L timeout -s KILL ${PASS_TIMEOUT:-120} rocprofv3 --pmc $PMC -d $out -o p --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --secondary none > $out/stdout 2> $out/stderr
  rc=$?
  echo "$L rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/stderr; exit $rc; fi
done
