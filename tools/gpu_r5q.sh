#!/bin/bash
# round 5: lane-refill K2 walk (VCT_K2_POOLW waves; 0 = one lane per voxel) -- parity, then times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_inject_bitexact_coarse_bricks tests/test_parity_gpu.py::test_voxelize_inject_mips_bitexact \
  tests/test_parity_gpu.py::test_mips_relight_sparse_bitexact tests/test_dump.py tests/test_parity_full.py > gpurun_out/t_r5q.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5q.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/t_r5q.log | head; exit $rc; }
for n in 256 512; do
for sc in atrium courtyard; do
  for pw in 0 1024 2048 3072 4096 8192 0 2048; do
    VCT_K2_POOLW=$pw timeout -k 10 120 python tools/k2_bench.py --scene $sc --n $n > gpurun_out/k2q_${n}_${sc}_$pw.log 2>&1 || { tail -3 gpurun_out/k2q_${n}_${sc}_$pw.log; exit 1; }
    echo "k2 $n $sc poolw=$pw: $(tail -1 gpurun_out/k2q_${n}_${sc}_$pw.log)"
  done
done
done
