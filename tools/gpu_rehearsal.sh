#!/bin/bash
# N-rank rehearsal of bench.py's default command on ONE GPU (gloo process group, every
# rank on cuda:0; RCCL refuses two ranks per device), timed against the driver's 600 s
# bench limit; then the per-rank K4 split measured on the one GPU (tools/rank_emul.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
N=${N:-8}
t0=$(date +%s)
VCT_DIST_BACKEND=gloo timeout -k 10 ${LIMIT:-600} python bench.py --gpus $N > gpurun_out/gloo$N.json 2> gpurun_out/gloo$N.err
rc=$?
echo "gloo $N ranks: rc=$rc in $(( $(date +%s) - t0 )) s"; head -c 400 gpurun_out/gloo$N.json; echo; tail -4 gpurun_out/gloo$N.err
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_EMUL" ] && exit 0
timeout -k 10 300 python tools/rank_emul.py --worlds 1,2,4,8 > gpurun_out/rank_emul.json 2> gpurun_out/rank_emul.err
echo "rank_emul rc=$?"; cat gpurun_out/rank_emul.json
