#!/bin/bash
# Both timed K4 forms (variant bits 0x1000000 union / 0x2000000 occupancy) of several
# builds, alternating builds in separate processes: LIBS="a.so b.so" bash tools/ab_forms.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=voxel-based-global-illumination_amd/vct
for r in $(seq 1 ${ROUNDS:-2}); do
  for sc in ${SCENES:-atrium courtyard}; do
    for lib in $LIBS; do
      VCT_LIB=$L/$lib timeout -k 10 200 python tools/ab.py --scene $sc --variants 0x1000000,0x2000000 --rounds 4 ${AB_ARGS:-} > gpurun_out/abf_$lib.json 2>&1 || { tail -5 gpurun_out/abf_$lib.json; exit 1; }
      echo "$sc $lib $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/abf_$lib.json').read().split('\n',1)[1] if open('gpurun_out/abf_$lib.json').read().startswith('/opt') else open('gpurun_out/abf_$lib.json').read()); print(' '.join(f\"{k}:{v['median_ms']}:{v['bitexact_vs_first']}\" for k,v in d['variants'].items()), d['steps'])")"
    done
  done
done
