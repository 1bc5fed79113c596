#!/bin/bash
# round 5: frames in flight per rank -- two vs three trace streams (rank emulation)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 2 3 2 3; do
  timeout -k 10 300 python tools/rank_emul.py --worlds 1,2,4,8 --reps 9 --streams $S > gpurun_out/rank_s$S.json 2> gpurun_out/rank_s$S.err || { tail -5 gpurun_out/rank_s$S.err; exit 1; }
  echo "streams $S: $(python -c "import json;d=json.load(open('gpurun_out/rank_s$S.json'));print({w:(x['k4_ms_max_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
