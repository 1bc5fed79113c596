#!/bin/bash
# Alternate tools/ab.py (variant 0) over several builds of libvct_hip.so, one process
# each, R rounds: ab_many.sh R a.so b.so c.so ...  (AB_ARGS passed to ab.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$1; shift
for r in $(seq 1 $R); do
  for L in "$@"; do
    VCT_LIB=$L timeout -k 10 200 python tools/ab.py --variants 0 --rounds 5 ${AB_ARGS:-} > gpurun_out/ab_lib.json 2>&1 || { tail -5 gpurun_out/ab_lib.json; exit 1; }
    echo "$(basename $L) $(grep -m1 median gpurun_out/ab_lib.json)"
  done
done
