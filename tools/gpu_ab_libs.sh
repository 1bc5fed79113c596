#!/bin/bash
# K4 A/B on one box: path counters of a debug build (DBG_LIB), then tools/ab_libs_n.sh over $LIBS
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
L=voxel-based-global-illumination_amd/vct
if [ -n "$DBG_LIB" ]; then
  for sc in ${DBG_SCENES:-atrium}; do
    VCT_DBG_LIB=$L/$DBG_LIB timeout -k 10 150 python tools/dbg_counters.py --scene $sc > gpurun_out/dbg_${DBG_LIB}_$sc.txt 2>&1 || { tail -5 gpurun_out/dbg_${DBG_LIB}_$sc.txt; exit 1; }
    grep -v amdgpu.ids gpurun_out/dbg_${DBG_LIB}_$sc.txt | head -12
  done
fi
[ -n "$LIBS" ] || exit 0
LIBS="$LIBS" ROUNDS=${ROUNDS:-2} AB_ARGS="${AB_ARGS:---variants 0x6000000,0x5000000}" bash tools/ab_libs_n.sh
