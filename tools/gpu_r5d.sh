#!/bin/bash
# round 5: reorder keys for G_rand (libs rk1 / rk2 vs the default), alternating processes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=voxel-based-global-illumination_amd/vct
for lib in libvct_hip.so libvct_hip_rk1.so libvct_hip_rk2.so; do
  VCT_LIB=$L/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "tests/test_parity_gpu.py::test_reorder_equals_screen_order" > gpurun_out/t_$lib.log 2>&1
  rc=$?; echo "parity $lib: $(tail -1 gpurun_out/t_$lib.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for lib in libvct_hip.so libvct_hip_rk1.so libvct_hip_rk2.so; do
    VCT_LIB=$L/$lib timeout -k 10 200 python tools/ab.py --variants 0x1008000,0x2008000 --rounds 3 --gbuffer rand > gpurun_out/ab_$lib.json 2>&1 || { tail -5 gpurun_out/ab_$lib.json; exit 1; }
    echo "rand $lib $(python -c "import json;d=json.load(open('gpurun_out/ab_$lib.json'));print({k:v['median_ms'] for k,v in d['variants'].items()})")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rand -o rand --output-format csv -- python3 tools/ab.py --variants 0x1008000 --rounds 2 --gbuffer rand > gpurun_out/prof_rand.log 2>&1
echo "rocprof rc=$?"
find gpurun_out/prof_rand -name "*kernel_stats.csv" -exec cp {} gpurun_out/rand_kernel_stats.csv \;
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/rand_kernel_stats.csv')):
    print(r['Name'][:90], r['Calls'], r['AverageNs'])
" | head -20
rm -rf gpurun_out/prof_rand
