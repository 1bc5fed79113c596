#!/bin/bash
# K2 A/B of two libraries (VCT_LIB), alternating processes: tools/k2_bench.py per scene and grid
cd "${GRAFT_REPO_ROOT:-/root/repo}"; L=voxel-based-global-illumination_amd/vct
for sc in atrium courtyard; do for n in 256 512; do for r in 1 2 3; do for lib in libvct_hip_k2base.so libvct_hip_k2chain.so; do
  VCT_LIB=$L/$lib timeout -k 10 120 python tools/k2_bench.py --scene $sc --n $n --reps 40 2>/dev/null | sed "s/^/$lib /" || exit 1
done; done; done; done
