#!/bin/bash
# Alternate tools/ab.py (variant 0) between two builds of libvct_hip.so in
# separate processes on the same box: ab_libs.sh <a.so> <b.so> [rounds]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in $(seq 1 ${3:-3}); do
  for L in "$1" "$2"; do
    VCT_LIB=$L timeout -k 10 200 python tools/ab.py --variants 0 --rounds 5 ${AB_ARGS:-} > gpurun_out/ab_lib.json 2>&1 || exit 1
    echo "$L $(grep -m1 median gpurun_out/ab_lib.json)"
  done
done
