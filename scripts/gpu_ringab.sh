#!/bin/bash
# GPU box: cfg2 A/B — fastchain (CVAE_RING=0) vs the ring chain (the default), alternating.
set -u
O=gpurun_out/ringab; mkdir -p $O
B="timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 400"
for i in 1 2; do
  CVAE_RING=0 $B > $O/fast$i.json 2> $O/fast$i.err && $B > $O/ring$i.json 2> $O/ring$i.err || { tail -5 $O/*.err; exit 1; }
done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernels_ms'],r.get('kernels_back_to_back_ms'))"; done
