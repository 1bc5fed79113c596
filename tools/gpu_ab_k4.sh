#!/bin/bash
# A/B of K4 library builds (tools/build_k4_variant.sh) on one box: parity subset, then
# alternating timings in the default form and the forced union form
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LIBS=${LIBS:-"libvct_hip_base.so libvct_hip_cov3n.so libvct_hip_cov2n.so"} ROUNDS=${ROUNDS:-2} SCENES=${SCENES:-atrium} timeout -k 10 600 bash tools/ab_libs_n.sh || exit $?
[ -n "$UNION" ] && LIBS=${LIBS:-"libvct_hip_base.so libvct_hip_cov3n.so libvct_hip_cov2n.so"} PARITY=0 ROUNDS=1 SCENES=atrium AB_ARGS="--variants 0x1000000" timeout -k 10 400 bash tools/ab_libs_n.sh
exit 0
