#!/bin/bash
# round 5: whole 1080p frames in flight -- two vs three trace streams
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 2 3 2 3; do
  timeout -k 10 300 python tools/rank_emul.py --worlds 1 --reps 9 --streams $S --overlap1 > gpurun_out/rank1_s$S.json 2> gpurun_out/rank1_s$S.err || { tail -5 gpurun_out/rank1_s$S.err; exit 1; }
  echo "streams $S: $(python -c "import json;d=json.load(open('gpurun_out/rank1_s$S.json'));print({w:(x['k4_ms_max_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
