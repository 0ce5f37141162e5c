#!/bin/bash
# round 5, timing only: the dW launch with the tail workgroups on half the batch (CVAE_DIAG_HALFK; the
# results are wrong) — what splitting the 24 doubled CUs' second tiles could buy
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05z}; mkdir -p $O
B="timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-b2b"
for r in 1 2; do
  for v in def hk256 hk232; do
    L=""; [ $v != def ] && L=$GRAFT_REPO_ROOT/build/ab/$v.so
    CVAE_LIB=$L $B > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -3 $O/${v}_$r.err; exit 1; }
  done
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
