#!/bin/bash
# A/B (round 6): the wide chain's ring depth (CVAE_WIDE_RING; base = 12), build/dx/wring*.so,
# cfg5 fp8 and bf16 at 100 steps, alternating
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06wr; mkdir -p $O
for i in 1 2; do
  for v in base wring10 wring14 wring16; do
    L=""; [ $v != base ] && L="CVAE_LIB=$PWD/build/dx/$v.so"
    env $L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/wfp8_${v}_$i.json 2> $O/wfp8_${v}_$i.err || exit 1
    env $L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 100 --warmup 10 --workload wide > $O/wbf16_${v}_$i.json 2> $O/wbf16_${v}_$i.err || exit 1
  done
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
