#!/bin/bash
# round 5: specular reorder key with normal bits (sn1: aperture, sign(n.z), 15-bit cell; sn3: aperture,
# octant, 15-bit cell) against the shipped aperture + 18-bit cell, G_rand, alternating processes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=voxel-based-global-illumination_amd/vct
for lib in libvct_hip.so libvct_hip_sn1.so libvct_hip_sn3.so libvct_hip.so libvct_hip_sn1.so libvct_hip_sn3.so; do
  VCT_LIB=$V/$lib timeout -k 10 200 python tools/ab.py --variants 0,0x1008000 --rounds 3 --gbuffer rand 2>/dev/null > gpurun_out/ab_y_$lib.json || exit 1
  echo "rand $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_y_$lib.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
done
