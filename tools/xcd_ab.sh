#!/bin/bash
# K4 workgroup -> XCD map variants (vct_variants.h bits 16-19) re-measured on the current kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for sc in atrium courtyard; do
  timeout -k 10 300 python tools/ab.py --variants 0,0x10000,0x30000,0x40000,0x60000 --rounds 5 --scene $sc > gpurun_out/xcd_$sc.json 2> gpurun_out/xcd_$sc.err || { tail -5 gpurun_out/xcd_$sc.err; exit 1; }
  echo "== $sc"; cat gpurun_out/xcd_$sc.json
done
