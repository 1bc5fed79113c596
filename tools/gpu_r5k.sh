#!/bin/bash
# round 5: the LPT size / overlap rule -- parity, then rank emulation (each rank's single launch
# and overlapped frames back to back) with the rule and with LPT off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_longest_first_dispatch_bitexact tests/test_parity_gpu.py::test_trace_variants_bitexact \
  tests/test_parity_gpu.py::test_frame_pipeline_equals_full_frames tests/test_parity_gpu.py::test_empty_space_maps_exact > gpurun_out/t_r5k.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5k.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/t_r5k.log | head; exit $rc; }
for v in 0 0x20000000 0x10000000; do
  timeout -k 10 300 python tools/rank_emul.py --worlds 1,2,4,8 --reps 9 --variant $v > gpurun_out/rank_k_$v.json 2> gpurun_out/rank_k_$v.err || { tail -5 gpurun_out/rank_k_$v.err; exit 1; }
  echo "ranks $v: $(python -c "import json;d=json.load(open('gpurun_out/rank_k_$v.json'));print({w:(x['k4_ms_max_rank'], x['k4_ms_min_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
