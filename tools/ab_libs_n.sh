#!/bin/bash
# A/B of several builds of libvct_hip.so, alternating in separate processes on one box:
#   LIBS="a.so b.so c.so" ROUNDS=3 AB_ARGS="--scene courtyard" bash tools/ab_libs_n.sh
# Each library first runs the K4 parity subset (PARITY=1, default) once.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=voxel-based-global-illumination_amd/vct
if [ "${PARITY:-1}" = 1 ]; then
  for lib in $LIBS; do
    VCT_LIB=$L/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      "tests/test_parity_gpu.py::test_trace_parity" "tests/test_parity_gpu.py::test_trace_variants_bitexact" \
      "tests/test_parity_gpu.py::test_trace_edge_cases" tests/test_parity_full.py > gpurun_out/t_$lib.log 2>&1
    rc=$?; echo "parity $lib: $(tail -1 gpurun_out/t_$lib.log)"; [ $rc -eq 0 ] || exit $rc
  done
fi
for sc in ${SCENES:-atrium courtyard}; do
  for r in $(seq 1 ${ROUNDS:-2}); do
    for lib in $LIBS; do
      VCT_LIB=$L/$lib timeout -k 10 200 python tools/ab.py --variants 0 --rounds 5 --scene $sc ${AB_ARGS:-} > gpurun_out/ab_$lib.json 2>&1 || { tail -5 gpurun_out/ab_$lib.json; exit 1; }
      echo "$sc $lib $(python3 tools/ab_summary.py gpurun_out/ab_$lib.json)"
    done
  done
done
