#!/bin/bash
# A/B several builds of libvct_hip.so (variant 0, tools/ab.py) in separate processes,
# alternating: ab_multi.sh <rounds> <lib.so>...   (AB_ARGS: extra ab.py arguments)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$1; shift
for r in $(seq 1 $R); do
  for L in "$@"; do
    VCT_LIB=$L timeout -k 10 200 python tools/ab.py --variants 0 --rounds 5 ${AB_ARGS:-} > gpurun_out/ab_m.json 2>&1 || exit 1
    echo "$(basename $L) $(grep -m1 median gpurun_out/ab_m.json)"
  done
done
