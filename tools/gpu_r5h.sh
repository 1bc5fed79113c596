#!/bin/bash
# round 5: path counters of G_rand's specular cone, one order vs the aperture-keyed order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in 0x1008000 0x41008000 0x5000000; do
  timeout -k 10 200 python tools/dbg_counters.py --gbuffer rand --nd 9 --spec 1 --variants $v > gpurun_out/dbg_rand_spec_$v.txt 2>&1 || { tail -5 gpurun_out/dbg_rand_spec_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/dbg_rand_spec_$v.txt
done
