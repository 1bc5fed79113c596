#!/bin/bash
# Union-form A/B on one box: the K4 parity subset with the product library, path counters
# of two debug builds with the union form forced, then the timed libraries alternating in
# separate processes over the workloads the union form serves (courtyard, G_rand, C5).
#   DBG_LIBS="libvct_hip_dbga.so libvct_hip_dbgb.so" LIBS="a.so b.so" bash tools/gpu_ab_union.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
L=voxel-based-global-illumination_amd/vct
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    "tests/test_parity_gpu.py::test_trace_parity" "tests/test_parity_gpu.py::test_trace_variants_bitexact" \
    "tests/test_parity_gpu.py::test_trace_edge_cases" tests/test_parity_full.py > gpurun_out/u_parity.log 2>&1
  rc=$?; echo "parity: $(tail -1 gpurun_out/u_parity.log)"; [ $rc -eq 0 ] || exit $rc
fi
for lib in $DBG_LIBS; do
  for w in "courtyard scene 0x1000000" "atrium rand 0x1008000"; do
    set -- $w
    VCT_DBG_LIB=$L/$lib timeout -k 10 150 python tools/dbg_counters.py --scene $1 --gbuffer $2 --variants $3 \
      > gpurun_out/udbg_${lib}_$2.txt 2>&1 || { tail -5 gpurun_out/udbg_${lib}_$2.txt; exit 1; }
    echo "== $lib $1 $2 $3"; grep -v amdgpu.ids gpurun_out/udbg_${lib}_$2.txt | head -8
  done
done
[ -n "$LIBS" ] || exit 0
run() {   # tag, ab.py args
  for r in $(seq 1 ${ROUNDS:-2}); do
    for lib in $LIBS; do
      VCT_LIB=$L/$lib timeout -k 10 300 python tools/ab.py --rounds 5 "${@:2}" > gpurun_out/uab_$lib.json 2>&1 || { tail -5 gpurun_out/uab_$lib.json; exit 1; }
      echo "$1 $lib $(python3 tools/ab_summary.py gpurun_out/uab_$lib.json)"
    done
  done
}
run courtyard --scene courtyard --variants 0x1000000,0
run G_rand --scene atrium --gbuffer rand --variants 0x1008000,0
run atrium --scene atrium --variants 0x1000000
[ "${C5:-1}" = 1 ] && run C5 --scene courtyard --n 512 --w 3840 --h 2160 --nd 16 --reps 2 --variants 0x1000000
exit 0
