#!/bin/bash
# alternating A/B: base vs build/dx/$V at wide fp8 (100 steps), wide bf16 and cfg2 (200 steps)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG}; mkdir -p $O
for i in 1 2; do
  for v in base $V; do
    L=""; [ $v != base ] && L="CVAE_LIB=$PWD/build/dx/$v.so"
    env $L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/wfp8_${v}_$i.json 2> $O/wfp8_${v}_$i.err || exit 1
    env $L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 100 --warmup 10 --workload wide > $O/wbf16_${v}_$i.json 2> $O/wbf16_${v}_$i.err || exit 1
    env $L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 200 --warmup 20 > $O/cfg2_${v}_$i.json 2> $O/cfg2_${v}_$i.err || exit 1
  done
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
