#!/bin/bash
# A/B of one library under two environments (separate processes, alternating):
#   LIB=libvct_hip_big.so ENVA="" ENVB="VCT_K4_BIG_OFF=1" ROUNDS=2 bash tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=voxel-based-global-illumination_amd/vct
for sc in ${SCENES:-atrium courtyard}; do
  for r in $(seq 1 ${ROUNDS:-2}); do
    for e in "$ENVA" "$ENVB"; do
      env $e VCT_LIB=$L/$LIB timeout -k 10 200 python tools/ab.py --rounds 5 --scene $sc ${AB_ARGS:---variants 0x6000000,0x5000000} > gpurun_out/abe.json 2>&1 || { tail -5 gpurun_out/abe.json; exit 1; }
      echo "$sc [$e] $(python3 tools/ab_summary.py gpurun_out/abe.json)"
    done
  done
done
