#!/bin/bash
# round 5: class-major reorder keys under super-cells (the top 3 / 6 / 9 Morton bits above the
# class) against fully class-major, G_rand, alternating processes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=voxel-based-global-illumination_amd/vct
for lib in libvct_hip_sc9.so libvct_hip_sc12.so libvct_hip_sc15.so libvct_hip_sc9.so libvct_hip_sc12.so libvct_hip_sc15.so; do
  VCT_LIB=$V/$lib timeout -k 10 200 python tools/ab.py --variants 0,0x1008000 --rounds 3 --gbuffer rand 2>/dev/null > gpurun_out/ab_z2_$lib.json || exit 1
  echo "rand $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_z2_$lib.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
done
