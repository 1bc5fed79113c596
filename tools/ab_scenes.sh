#!/bin/bash
# Alternate tools/ab.py between builds of libvct_hip.so, per scene, in separate
# processes on one box; one compact line per run (median ms of each variant):
#   ROUNDS=2 SCENES="atrium courtyard" VARIANTS=0x6000000,0x5000000 ab_scenes.sh <a.so> <b.so> [<c.so> ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for sc in ${SCENES:-atrium courtyard}; do
    for L in "$@"; do
      VCT_LIB=$L timeout -k 10 200 python tools/ab.py --variants ${VARIANTS:-0x6000000,0x5000000} --rounds 5 \
          --scene $sc ${AB_ARGS:-} > gpurun_out/ab_scene.json 2> gpurun_out/ab_scene.err || { tail -5 gpurun_out/ab_scene.err; exit 1; }
      python3 - "$L" "$sc" <<'EOF'
import json, sys
d = json.load(open("gpurun_out/ab_scene.json"))
print(sys.argv[2], sys.argv[1].rsplit("/", 1)[-1],
      " ".join(f"{k}:{v['median_ms']}{'' if v['bitexact_vs_first'] else '(DIFF)'}" for k, v in d["variants"].items()))
EOF
    done
  done
done
