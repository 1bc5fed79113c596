#!/bin/bash
# round 5: the level-A brick test's forms (zb0 per-lane D2 test, zb1 scalar D3 test with
# overlapped stagings, zb2 scalar test in the old order, zb3 scalar pre-filter + D2), path
# counters of zb0 / zb1, and the K2 shade / fused-walk switches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=voxel-based-global-illumination_amd/vct
for sc in atrium courtyard; do
  for lib in zb0 zb2 zb3 zb0 zb2 zb3; do
    VCT_LIB=$V/libvct_hip_$lib.so timeout -k 10 200 python tools/ab.py --variants 0 --rounds 5 --scene $sc 2>/dev/null > gpurun_out/ab_zbj_${sc}_$lib.json || exit 1
    echo "$sc $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_zbj_${sc}_$lib.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
  done
done
for z in 0 1; do
  VCT_DBG_LIB=$V/libvct_hip_dbgz$z.so timeout -k 10 200 python tools/dbg_counters.py --variants 0x2000000 > gpurun_out/dbg_zb$z.txt 2>&1 || { tail -5 gpurun_out/dbg_zb$z.txt; exit 1; }
  echo "== dbg zb$z"; grep -v amdgpu.ids gpurun_out/dbg_zb$z.txt | head -60
done
for sc in atrium courtyard; do
  for sj in 16 4 1 0 16 0; do
    VCT_K2_SHADEJ=$sj timeout -k 10 120 python tools/k2_bench.py --scene $sc > gpurun_out/k2j_${sc}_$sj.log 2>&1 || { tail -3 gpurun_out/k2j_${sc}_$sj.log; exit 1; }
    echo "k2 $sc shadej=$sj: $(tail -1 gpurun_out/k2j_${sc}_$sj.log)"
  done
done
