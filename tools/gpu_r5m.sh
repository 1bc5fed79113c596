#!/bin/bash
# round 5: cone-part splits at 2 / 4 / 8 ranks with longest-first dispatch on
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "2,4:0x400" "2,4:0" "8:0x300400" "8:0x400400" "8:0" "4:0x300400" "4:0x400"; do
  w=${spec%%:*}; v=${spec##*:}
  timeout -k 10 300 python tools/rank_emul.py --worlds $w --reps 9 --variant $v > gpurun_out/rank_m_${w/,/_}_$v.json 2> gpurun_out/rank_m_${w/,/_}_$v.err || { tail -5 gpurun_out/rank_m_${w/,/_}_$v.err; exit 1; }
  echo "ranks $w $v: $(python -c "import json;d=json.load(open('gpurun_out/rank_m_${w/,/_}_$v.json'));print({w:(x['k4_ms_max_rank'], x['k4_ms_min_rank'], x.get('k4_ms_per_frame_overlapped_max_rank')) for w,x in d.items()})")"
done
