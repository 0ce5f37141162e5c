#!/bin/bash
# A/B (round 6): cfg5 fp8 with 0-4 of each wave's 4 eps draws in the prologue (CVAE_DIAG_EPS_PRO_F8;
# base = 2), build/dx/eps*.so, 100 steps, alternating
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06eps; mkdir -p $O
for i in 1 2; do
  for v in base eps0 eps1 eps3 eps4; do
    L=""; [ $v != base ] && L="CVAE_LIB=$PWD/build/dx/$v.so"
    env $L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/wfp8_${v}_$i.json 2> $O/wfp8_${v}_$i.err || exit 1
  done
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
