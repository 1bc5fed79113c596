#!/bin/bash
# The round's GPU evidence for the shipped library, on one box:
#   1. the GPU suite (pytest -m gpu);
#   2. tools/gpu_final.sh: the default bench line (CPU baseline included), a rocprofv3
#      kernel trace + stats of the same command, smoke();
#   3. K4 path counters and phase clocks of the metric workload (debug / clock builds);
#   4. the metric workload's kernel trace with overlap off (tools/gpu_trace_c3.sh);
#   5. the PMC records of every bench line (tools/pmc_all.sh).
#   TAG=r6a bash tools/gpu_evidence.sh        (outputs under gpurun_out/, tagged)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6}
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo "pytest: $(tail -1 gpurun_out/pytest_gpu_$T.log)"; [ $rc -eq 0 ] || exit $rc
TAG=$T bash tools/gpu_final.sh || exit $?
for mode in "" "--clk"; do
  timeout -k 10 200 python tools/dbg_counters.py $mode > gpurun_out/dbg_$T${mode/--/_}.txt 2>&1 || { tail -5 gpurun_out/dbg_$T${mode/--/_}.txt; exit 1; }
  echo "== dbg $mode"; grep -v amdgpu.ids gpurun_out/dbg_$T${mode/--/_}.txt | head -20
done
[ -n "$SKIP_PMC" ] && exit 0
TAG=${T}c bash tools/gpu_trace_c3.sh > gpurun_out/trace_c3_$T.log 2>&1 || { tail gpurun_out/trace_c3_$T.log; exit 1; }
head -3 gpurun_out/trace_c3_$T.log
TAG=${T}p PASS_TIMEOUT=200 bash tools/pmc_all.sh > gpurun_out/pmc_$T.log 2>&1; rc=$?; tail -3 gpurun_out/pmc_$T.log; exit $rc
