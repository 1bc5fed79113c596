#!/bin/bash
# round 5: longest-first dispatch -- parity, then A/B (on / off) on the C3 frame, the
# courtyard, G_rand and the 2 / 4 / 8-rank launches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_longest_first_dispatch_bitexact tests/test_parity_gpu.py::test_trace_variants_bitexact \
  tests/test_parity_gpu.py::test_frame_pipeline_equals_full_frames tests/test_parity_gpu.py::test_reorder_equals_screen_order \
  tests/test_parity_gpu.py::test_reordered_frames_overlapped tests/test_parity_gpu.py::test_trace_form_tuner \
  tests/test_parity_gpu.py::test_tiled_trace_equals_full_frame tests/test_parity_gpu.py::test_multi_device_context \
  tests/test_parity_gpu.py::test_inject_bitexact_coarse_bricks tests/test_parity_gpu.py::test_voxelize_inject_mips_bitexact \
  tests/test_parity_gpu.py::test_mips_relight_sparse_bitexact tests/test_dump.py \
  tests/test_parity_full.py > gpurun_out/t_r5f.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5f.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/t_r5f.log | head; exit $rc; }
for sc in atrium courtyard; do
  for sk in 1 0 1 0; do
    VCT_K2_SKIP=$sk timeout -k 10 120 python tools/k2_bench.py --scene $sc > gpurun_out/k2_${sc}_${sk}.log 2>&1 || { tail -3 gpurun_out/k2_${sc}_${sk}.log; exit 1; }
    echo "k2 $sc skip=$sk: $(tail -1 gpurun_out/k2_${sc}_${sk}.log)"
  done
  timeout -k 10 300 python tools/ab.py --variants 0,0x20000000 --rounds 7 --scene $sc 2>/dev/null > gpurun_out/ab_lpt_$sc.json || exit 1
  echo "$sc: $(python -c "import json;d=json.load(open('gpurun_out/ab_lpt_$sc.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
done
timeout -k 10 300 python tools/ab.py --variants 0,0x20000000,0x40000000,0x1008000,0x41008000 --rounds 3 --gbuffer rand 2>/dev/null > gpurun_out/ab_lpt_rand.json || exit 1
echo "rand: $(python -c "import json;d=json.load(open('gpurun_out/ab_lpt_rand.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
for v in 0 0x20000000; do
  timeout -k 10 300 python tools/rank_emul.py --worlds 1,2,4,8 --reps 9 --variant $v > gpurun_out/rank_lpt_$v.json 2> gpurun_out/rank_lpt_$v.err || { tail -5 gpurun_out/rank_lpt_$v.err; exit 1; }
  echo "ranks $v: $(python -c "import json;d=json.load(open('gpurun_out/rank_lpt_$v.json'));print({w:(x['k4_ms_max_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
timeout -k 10 400 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --multi-config none > gpurun_out/bench_lpt.json 2> gpurun_out/bench_lpt.err || { tail -5 gpurun_out/bench_lpt.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_lpt.json'));print('bench', d['value'], d['ms_per_step'], d['k4_kernel_ms_avg'], d['secondary']['k4_kernel_ms_avg'], d['stress']['default_ms'])"
for v in 0x300400 0x500400 0x900400 0x1000000 0x2000000 0x1300400 0x2300400; do
  timeout -k 10 200 python tools/rank_emul.py --worlds 8 --reps 9 --variant $v > gpurun_out/rank8_lpt_$v.json 2> gpurun_out/rank8_lpt_$v.err || { tail -5 gpurun_out/rank8_lpt_$v.err; exit 1; }
  echo "rank8 $v: $(python -c "import json;d=json.load(open('gpurun_out/rank8_lpt_$v.json'));print({w:(x['k4_ms_max_rank'], x['k4_ms_min_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
