#!/bin/bash
# GPU call body: K4 parity tests with the working-tree library, then A/B of
# base vs working tree on the atrium and the courtyard (tools/ab_libs.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=voxel-based-global-illumination_amd/vct
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_parity_gpu.py::test_trace_parity" "tests/test_parity_gpu.py::test_trace_variants_bitexact" "tests/test_parity_gpu.py::test_trace_edge_cases" "tests/test_parity_gpu.py::test_tiled_trace_equals_full_frame" tests/test_parity_full.py > gpurun_out/t.log 2>&1
rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh $L/libvct_hip_base.so $L/libvct_hip.so ${ROUNDS:-2} || exit 1
AB_ARGS="--scene courtyard" bash tools/ab_libs.sh $L/libvct_hip_base.so $L/libvct_hip.so ${ROUNDS:-2}
