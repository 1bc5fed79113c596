#!/bin/bash
# round 5 final evidence for the shipped library: GPU suite, bench line + rocprofv3 trace +
# smoke + path counters / phase clocks (tools/gpu_r5_final.sh), the metric workload's kernel
# trace with overlap off (tools/gpu_trace_c3.sh) and the PMC records of every line
# (tools/pmc_all.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo "pytest: $(tail -1 gpurun_out/pytest_gpu_$T.log)"; [ $rc -eq 0 ] || exit $rc
TAG=$T bash tools/gpu_r5_final.sh || exit $?
TAG=${T}c bash tools/gpu_trace_c3.sh > gpurun_out/trace_c3_$T.log 2>&1 || { tail gpurun_out/trace_c3_$T.log; exit 1; }
head -3 gpurun_out/trace_c3_$T.log
TAG=${T}p PASS_TIMEOUT=200 bash tools/pmc_all.sh > gpurun_out/pmc_$T.log 2>&1; rc=$?; tail -3 gpurun_out/pmc_$T.log; exit $rc
