#!/bin/bash
# round 5: more reorder key forms under super-cells (tq15: quarter-octave apertures over 15-bit cells;
# t3s18: octave apertures; dO18: diffuse octant-major over 18-bit cells), G_rand, alternating processes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=voxel-based-global-illumination_amd/vct
for lib in libvct_hip_tq15.so libvct_hip_te15.so libvct_hip_tq15s6.so libvct_hip_tq15.so libvct_hip_te15.so libvct_hip_tq15s6.so; do
  VCT_LIB=$V/$lib timeout -k 10 200 python tools/ab.py --variants 0,0x1008000 --rounds 3 --gbuffer rand 2>/dev/null > gpurun_out/ab_ab_$lib.json || exit 1
  echo "rand $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_ab_$lib.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
done
