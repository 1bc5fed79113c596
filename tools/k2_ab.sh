#!/bin/bash
# K2 A/B between builds of libvct_hip.so, alternating in separate processes on one box:
#   tools/k2_ab.sh <a.so> <b.so> ... (ROUNDS, SCENES, N from the environment)
# Each line: library, tools/k2_bench.py's ms per inject and its level-0 hash (the builds
# must agree bit for bit).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for sc in ${SCENES:-atrium courtyard}; do
    for L in "$@"; do
      out=$(VCT_LIB=$L timeout -k 10 120 python tools/k2_bench.py --scene $sc --n ${N:-256} --reps ${REPS:-50} 2>&1) || { echo "$out" | tail -5; exit 1; }
      echo "$(basename $L) $out"
    done
  done
done
