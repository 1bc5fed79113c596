#!/bin/bash
# One GPU call: parity tests, then (only if nothing faulted) a short bench.
# Stops at the first fault / abort / timeout (exit codes other than 0 and 1, or a
# runtime fault message in the log).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
faulted() { grep -qE "HSA_STATUS_ERROR|Memory access fault|APERTURE_VIOLATION|GPU core dump" "$@"; }
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if faulted gpurun_out/pytest_gpu.log; then echo "GPU FAULT in tests"; exit 99; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
echo "bench rc=$brc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
if faulted gpurun_out/bench.err; then echo "GPU FAULT in bench"; exit 99; fi
if [ $brc -ne 0 ]; then exit $brc; fi
# extra bench configurations: EXTRA="args1;args2"
if [ -n "$EXTRA" ]; then
  IFS=';' read -ra XS <<< "$EXTRA"
  i=0
  for xa in "${XS[@]}"; do
    i=$((i+1))
    timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --no-cpu-baseline $xa > gpurun_out/bench_x$i.json 2> gpurun_out/bench_x$i.err
    xrc=$?
    echo "extra[$i] ($xa) rc=$xrc"; cat gpurun_out/bench_x$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['k4_kernel_ms_avg'], d['roofline']['frac'])" 2>/dev/null
    if faulted gpurun_out/bench_x$i.err; then echo "GPU FAULT in extra bench"; exit 99; fi
    if [ $xrc -ne 0 ]; then tail -5 gpurun_out/bench_x$i.err; exit $xrc; fi
  done
fi
exit 0
