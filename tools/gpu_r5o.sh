#!/bin/bash
# round 5: K4 with ConeCtl packed into one SGPR (libvct_hip.so) against the unpacked build
# (libvct_hip_base.so), alternating processes; parity first
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_trace_variants_bitexact tests/test_parity_gpu.py::test_empty_space_maps_exact \
  tests/test_parity_full.py > gpurun_out/t_r5o.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5o.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/t_r5o.log | head; exit $rc; }
V=voxel-based-global-illumination_amd/vct
for sc in atrium courtyard; do
  for lib in libvct_hip_base.so libvct_hip.so libvct_hip_base.so libvct_hip.so; do
    VCT_LIB=$V/$lib timeout -k 10 200 python tools/ab.py --variants 0,0x1000000,0x2000000 --rounds 5 --scene $sc 2>/dev/null > gpurun_out/ab_o_${sc}_$lib.json || exit 1
    echo "$sc $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_o_${sc}_$lib.json'));print({k:v['median_ms'] for k,v in d['variants'].items()}, d['k4_form'])")"
  done
done
