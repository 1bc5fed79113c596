#!/bin/bash
# round 5: longest-first dispatch in stable bands vs a full sort vs off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_longest_first_dispatch_bitexact tests/test_parity_gpu.py::test_trace_variants_bitexact \
  tests/test_parity_gpu.py::test_frame_pipeline_equals_full_frames > gpurun_out/t_r5g.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5g.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/t_r5g.log | head; exit $rc; }
for sc in atrium courtyard; do
  timeout -k 10 300 python tools/ab.py --variants 0,0x80000000,0x20000000 --rounds 7 --scene $sc 2>/dev/null > gpurun_out/ab_lpt_$sc.json || exit 1
  echo "$sc: $(python -c "import json;d=json.load(open('gpurun_out/ab_lpt_$sc.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
done
for v in 0 0x20000000 0; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 4 --no-cpu-baseline --multi-config none --stress none --secondary none --variant $v > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err || { tail -5 gpurun_out/bench_v$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_v$v.json'));print('bench $v', d['value'], d['ms_per_step'], d['k4_kernel_ms_avg'], d['k4_dispatch'], d['frame_overlap'])"
done
for v in 0 0x20000000; do
  timeout -k 10 300 python tools/rank_emul.py --worlds 1,2,4,8 --reps 9 --variant $v > gpurun_out/rank_lpt_$v.json 2> gpurun_out/rank_lpt_$v.err || { tail -5 gpurun_out/rank_lpt_$v.err; exit 1; }
  echo "ranks $v: $(python -c "import json;d=json.load(open('gpurun_out/rank_lpt_$v.json'));print({w:(x['k4_ms_max_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
