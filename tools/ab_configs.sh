#!/bin/bash
# A/B of several builds over the BASELINE configurations (one process per build and config):
#   LIBS="a.so b.so" bash tools/ab_configs.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=voxel-based-global-illumination_amd/vct
CFGS=${CFGS:-"C1:--scene cornell --n 64 --w 1280 --h 720 --nd 1 --spec 0|C2:--n 128 --w 1280 --h 720 --spec 0|C3:|C4:--n 512 --w 3840 --h 2160|C5:--n 512 --w 3840 --h 2160 --scene courtyard --nd 16|Ccourt:--scene courtyard|Crand:--gbuffer rand --variants 0x8000"}
IFS='|' read -ra CS <<< "$CFGS"
for r in $(seq 1 ${ROUNDS:-1}); do
  for c in "${CS[@]}"; do
    name=${c%%:*}; args=${c#*:}
    for lib in $LIBS; do
      VCT_LIB=$L/$lib timeout -k 10 300 python tools/ab.py --variants ${VARIANT:-0} --rounds 3 --reps 3 $args > gpurun_out/abc_$lib.json 2>&1 || { tail -5 gpurun_out/abc_$lib.json; exit 1; }
      echo "$name $lib $(python3 tools/ab_summary.py gpurun_out/abc_$lib.json) $(grep -o '"k4_form": [-0-9a-z]*' gpurun_out/abc_$lib.json)"
    done
  done
done
