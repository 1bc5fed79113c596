#!/bin/bash
# round 5: K4 work-queue form (0x8000000) -- parity, the default's cost of the change (HEAD
# trace vs this one, alternating processes), rank emulation queue vs one unit per workgroup
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_trace_variants_bitexact tests/test_parity_gpu.py::test_tiled_trace_equals_full_frame \
  tests/test_parity_gpu.py::test_longest_first_dispatch_bitexact tests/test_parity_gpu.py::test_frame_pipeline_equals_full_frames > gpurun_out/t_r5l.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5l.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/t_r5l.log | head; exit $rc; }
V=voxel-based-global-illumination_amd/vct
for sc in atrium courtyard; do
  for lib in libvct_hip_head.so libvct_hip.so libvct_hip_head.so libvct_hip.so; do
    VCT_LIB=$V/$lib timeout -k 10 200 python tools/ab.py --variants 0,0x8000000 --rounds 5 --scene $sc 2>/dev/null > gpurun_out/ab_q_${sc}_$lib.json || exit 1
    echo "$sc $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_q_${sc}_$lib.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
  done
done
for v in 0 0x8000000 0x28000000; do
  timeout -k 10 300 python tools/rank_emul.py --worlds 1,2,4,8 --reps 9 --variant $v > gpurun_out/rank_q_$v.json 2> gpurun_out/rank_q_$v.err || { tail -5 gpurun_out/rank_q_$v.err; exit 1; }
  echo "ranks $v: $(python -c "import json;d=json.load(open('gpurun_out/rank_q_$v.json'));print({w:(x['k4_ms_max_rank'], x['k4_ms_min_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
