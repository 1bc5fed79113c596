#!/bin/bash
# round 5: K2 walk over brick-grouped occupancy words (VCT_K2_BB=1, default) vs the linear bitmask
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_inject_bitexact_coarse_bricks tests/test_parity_gpu.py::test_voxelize_inject_mips_bitexact \
  tests/test_parity_gpu.py::test_mips_relight_sparse_bitexact tests/test_dump.py tests/test_parity_full.py > gpurun_out/t_r5p.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5p.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/t_r5p.log | head; exit $rc; }
for sc in atrium courtyard; do
  for bb in 1 0 1 0; do
    VCT_K2_BB=$bb timeout -k 10 120 python tools/k2_bench.py --scene $sc > gpurun_out/k2p_${sc}_$bb.log 2>&1 || { tail -3 gpurun_out/k2p_${sc}_$bb.log; exit 1; }
    echo "k2 $sc bb=$bb: $(tail -1 gpurun_out/k2p_${sc}_$bb.log)"
  done
  for bb in 1 0; do
    VCT_K2_BB=$bb timeout -k 10 120 python tools/k2_bench.py --scene $sc --n 512 > gpurun_out/k2p512_${sc}_$bb.log 2>&1 || { tail -3 gpurun_out/k2p512_${sc}_$bb.log; exit 1; }
    echo "k2 512 $sc bb=$bb: $(tail -1 gpurun_out/k2p512_${sc}_$bb.log)"
  done
done
