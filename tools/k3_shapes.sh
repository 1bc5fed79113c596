#!/bin/bash
# K3 relight / full builds per block depth (tools/k3_bench.py), two rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
  for sc in atrium courtyard; do
    for n in 256 512; do
      for cfg in "VCT_K3_BZ=4" "VCT_K3_BZ=2" "VCT_K3_BZ=8" "VCT_K3_BZ=4 VCT_K3_SPARSE=0"; do
        env $cfg timeout -k 10 120 python tools/k3_bench.py --scene $sc --n $n --reps 20 2>/dev/null | grep K3 | sed "s/^/$cfg: /" || exit 1
      done
    done
  done
done
