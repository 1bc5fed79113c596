#!/bin/bash
# round 5: wave timelines of the full C3 frame, one vs two waves per workgroup (occupancy form)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in 0x12000000 0x2000000 0x1000000; do
  timeout -k 10 120 python tools/wave_sched.py --wv --parts 2 --slots 5120 --variant $v > gpurun_out/waves1_$v.json 2>&1 || { tail -5 gpurun_out/waves1_$v.json; exit 1; }
  echo "waves1 $v: $(tail -1 gpurun_out/waves1_$v.json)"
done
