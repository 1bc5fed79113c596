#!/bin/bash
# round 5 final evidence (one box): tools/gpu_final.sh (default bench line with the CPU
# baseline, rocprofv3 kernel trace + stats of the same command, smoke), then the K4 path
# counters and phase clocks of the metric workload (debug / clock builds)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r5} bash tools/gpu_final.sh || exit $?
for mode in "" "--clk"; do
  timeout -k 10 200 python tools/dbg_counters.py $mode > gpurun_out/dbg_final${mode/--/_}.txt 2>&1 || { tail -5 gpurun_out/dbg_final${mode/--/_}.txt; exit 1; }
  echo "== dbg $mode"; grep -v amdgpu.ids gpurun_out/dbg_final${mode/--/_}.txt | head -20
done
