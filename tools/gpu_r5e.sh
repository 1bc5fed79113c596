#!/bin/bash
# round 5: LPT dispatch oracle (8 / 4 ranks, full frame), G_rand cone-set split
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for wr in "8 0" "8 3" "4 0" "1 0"; do
  set -- $wr
  timeout -k 10 200 python tools/lpt_emul.py --world $1 --rank $2 > gpurun_out/lpt_$1_$2.json 2> gpurun_out/lpt_$1_$2.err || { tail -5 gpurun_out/lpt_$1_$2.err; exit 1; }
  echo "lpt $1/$2: $(cat gpurun_out/lpt_$1_$2.json)"
done
timeout -k 10 200 python tools/lpt_emul.py --world 8 --variant 0x902400 > gpurun_out/lpt_8_s9.json 2> gpurun_out/lpt_8_s9.err && echo "lpt 8 (9 parts, spec first): $(cat gpurun_out/lpt_8_s9.json)"
for cs in "--nd 9 --spec 0" "--nd 0 --spec 1" "--nd 9 --spec 1"; do
  timeout -k 10 200 python tools/ab.py --variants 0x1008000,0x2008000 --rounds 3 --gbuffer rand $cs 2>/dev/null > gpurun_out/ab_rand_cs.json || exit 1
  echo "rand $cs: $(python -c "import json;d=json.load(open('gpurun_out/ab_rand_cs.json'));print({k:v['median_ms'] for k,v in d['variants'].items()}, d['steps'])")"
done
