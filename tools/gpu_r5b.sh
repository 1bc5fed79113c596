#!/bin/bash
# round 5: two waves per workgroup (the occupancy form) -- parity subset, then A/B in one
# process (forced forms) on the atrium / courtyard / G_rand, and the 8-rank launch
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_trace_parity tests/test_parity_gpu.py::test_trace_variants_bitexact \
  tests/test_parity_gpu.py::test_trace_edge_cases tests/test_parity_gpu.py::test_occupancy_form_curved_bitexact \
  tests/test_parity_full.py > gpurun_out/t_r5b.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5b.log)"; [ $rc -eq 0 ] || exit $rc
for sc in atrium courtyard; do
  timeout -k 10 300 python tools/ab.py --variants 0x2000000,0x12000000,0x1000000,0 --rounds 5 --scene $sc > gpurun_out/ab_wpb_$sc.json 2>&1 || { tail -5 gpurun_out/ab_wpb_$sc.json; exit 1; }
  echo "$sc: $(python -c "import json;d=json.load(open('gpurun_out/ab_wpb_$sc.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
done
timeout -k 10 300 python tools/ab.py --variants 0x2008000,0x12008000,0x1008000 --rounds 3 --gbuffer rand > gpurun_out/ab_wpb_rand.json 2>&1 || { tail -5 gpurun_out/ab_wpb_rand.json; exit 1; }
echo "rand: $(python -c "import json;d=json.load(open('gpurun_out/ab_wpb_rand.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()})")"
for v in 0 0x10000000 0x2000000 0x12000000; do
  timeout -k 10 200 python tools/rank_emul.py --worlds 1,4,8 --reps 7 --variant $v > gpurun_out/rank_$v.json 2> gpurun_out/rank_$v.err || { tail -5 gpurun_out/rank_$v.err; exit 1; }
  echo "ranks variant $v: $(python -c "import json;d=json.load(open('gpurun_out/rank_$v.json'));print({w:(x['k4_ms_max_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
