#!/bin/bash
# K2 A/B between shadow-walk launches of one library (VCT_K2_WALK codes: segments * 1000000
# + cells per batch * 10000 + block threads), alternating in separate processes on one box:
#   WALKS="160256 2160256 4160256" ROUNDS=2 SCENES="atrium courtyard" NS="256 512" bash tools/k2_walk_ab.sh
# Each line: walk code, tools/k2_bench.py's ms per inject and its level-0 hash (every walk
# must give the same hash).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for n in ${NS:-256}; do
  for sc in ${SCENES:-atrium courtyard}; do
    for r in $(seq 1 ${ROUNDS:-2}); do
      for w in ${WALKS:-160256 2160256}; do
        out=$(VCT_K2_WALK=$w timeout -k 10 120 python tools/k2_bench.py --scene $sc --n $n --reps ${REPS:-50} 2>&1) || { echo "$out" | tail -5; exit 1; }
        echo "$w $(echo "$out" | grep -v amdgpu.ids)"
      done
    done
  done
done
