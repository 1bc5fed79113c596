#!/bin/bash
# round 5: five-face 4x4x3 staging in the union form -- parity (variants, full configs), then A/B
# against the previous trace (libvct_hip_pre5.so), alternating processes, courtyard and atrium
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py::test_trace_variants_bitexact tests/test_parity_gpu.py::test_empty_space_maps_exact \
  tests/test_parity_gpu.py::test_tiled_trace_equals_full_frame tests/test_parity_full.py > gpurun_out/t_r5ac.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/t_r5ac.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/t_r5ac.log | head; exit $rc; }
V=voxel-based-global-illumination_amd/vct
for sc in courtyard atrium; do
  for lib in libvct_hip_pre5.so libvct_hip.so libvct_hip_pre5.so libvct_hip.so; do
    VCT_LIB=$V/$lib timeout -k 10 200 python tools/ab.py --variants 0,0x1000000,0x2000000 --rounds 5 --scene $sc 2>/dev/null > gpurun_out/ab_ac_${sc}_$lib.json || exit 1
    echo "$sc $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_ac_${sc}_$lib.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
  done
done
for lib in libvct_hip_pre5.so libvct_hip.so; do
  VCT_LIB=$V/$lib timeout -k 10 300 python tools/ab.py --variants 0,0x1000000,0x2000000 --rounds 3 --scene courtyard --n 512 --w 3840 --h 2160 --nd 16 2>/dev/null > gpurun_out/ab_ac_c5_$lib.json || exit 1
  echo "c5 $lib: $(python -c "import json;d=json.load(open('gpurun_out/ab_ac_c5_$lib.json'));print({k:(v['median_ms'],v['bitexact_vs_first']) for k,v in d['variants'].items()}, d['k4_form'])")"
done
