#!/bin/bash
# round 5: K4 level-A brick test on the scalar unit (D3 maps) -- parity, then A/B against
# the per-lane test (libvct_hip_zb0.so) in alternating processes; the LPT size rule
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_empty_space_maps_exact tests/test_parity_gpu.py::test_trace_variants_bitexact \
  tests/test_parity_gpu.py::test_longest_first_dispatch_bitexact tests/test_parity_gpu.py::test_reorder_equals_screen_order \
  tests/test_parity_gpu.py::test_tiled_trace_equals_full_frame tests/test_parity_gpu.py::test_mips_relight_sparse_bitexact \
  tests/test_parity_full.py > gpurun_out/t_r5i.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5i.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/t_r5i.log | head; exit $rc; }
V=voxel-based-global-illumination_amd/vct
for sc in atrium courtyard; do
  for lib in libvct_hip.so libvct_hip_zb0.so libvct_hip.so libvct_hip_zb0.so; do
    VCT_LIB=$V/$lib timeout -k 10 200 python tools/ab.py --variants 0,0x1000000,0x2000000 --rounds 5 --scene $sc 2>/dev/null > gpurun_out/ab_zb_${sc}_$lib.json || exit 1
    echo "$sc $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_zb_${sc}_$lib.json'));print({k:v['median_ms'] for k,v in d['variants'].items()}, d['k4_form'])")"
  done
done
for lib in libvct_hip.so libvct_hip_zb0.so; do
  VCT_LIB=$V/$lib timeout -k 10 200 python tools/ab.py --variants 0 --rounds 3 --gbuffer rand 2>/dev/null > gpurun_out/ab_zb_rand_$lib.json || exit 1
  echo "rand $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_zb_rand_$lib.json'));print({k:v['median_ms'] for k,v in d['variants'].items()}, d['k4_form'])")"
done
timeout -k 10 300 python tools/rank_emul.py --worlds 1,4,8 --reps 9 > gpurun_out/rank_r5i.json 2> gpurun_out/rank_r5i.err || { tail -5 gpurun_out/rank_r5i.err; exit 1; }
echo "ranks: $(python -c "import json;d=json.load(open('gpurun_out/rank_r5i.json'));print({w:(x['k4_ms_max_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
