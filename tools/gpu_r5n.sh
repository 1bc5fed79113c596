#!/bin/bash
# round 5: rank emulation with the trace streams made once (order of world sizes 1,2,4,8 and 8,4,2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for ws in 1,2,4,8 8,4,2 4; do
  timeout -k 10 300 python tools/rank_emul.py --worlds $ws --reps 9 > gpurun_out/rank_n_${ws//,/_}.json 2> gpurun_out/rank_n_${ws//,/_}.err || { tail -5 gpurun_out/rank_n_${ws//,/_}.err; exit 1; }
  echo "ranks $ws: $(python -c "import json;d=json.load(open('gpurun_out/rank_n_${ws//,/_}.json'));print({w:(x['k4_ms_max_rank'], x['k4_ms_min_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
