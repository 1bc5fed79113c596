#!/bin/bash
# round 5 first GPU call: the gpu test suite + a short bench, then the 8-rank split
# experiments (per-rank launch times for cone-part layouts; wave timelines of rank 0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_BENCH=${SKIP_BENCH:-} bash tools/gpu_round.sh || exit $?
for v in 0 0x2400 0x502400 0x902400 0x900400; do
  timeout -k 10 200 python tools/rank_emul.py --worlds 8 --reps 7 --variant $v > gpurun_out/rank8_$v.json 2> gpurun_out/rank8_$v.err || { tail -5 gpurun_out/rank8_$v.err; exit 1; }
  echo "rank8 variant $v: $(python -c "import json;d=json.load(open('gpurun_out/rank8_$v.json'))['8'];print(d['k4_ms_max_rank'], d['k4_ms_min_rank'], d.get('k4_ms_per_frame_overlapped_max_rank'))")"
done
for v in 0 0x902400; do
  timeout -k 10 120 python tools/wave_sched.py --wv --world 8 --rank 0 --parts $([ $v = 0 ] && echo 3 || echo 10) --variant $v > gpurun_out/waves8_$v.json 2>&1 || { tail -5 gpurun_out/waves8_$v.json; exit 1; }
  echo "waves8 $v: $(cat gpurun_out/waves8_$v.json | tail -1)"
done
