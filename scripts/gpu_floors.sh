#!/bin/bash
# GPU box: row-chain floors — diagnostic builds without weight loads / arena stores / both (results
# are garbage; only the kernel times matter), fastchain (default) and the ring chain.
set -u
O=gpurun_out/floors; mkdir -p $O
B="timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 200"
for v in nowl nost both; do
  for ring in 0 1; do
    CVAE_RING=$ring CVAE_LIB=$PWD/build/diag/$v.so $B > $O/bench_${v}_r$ring.json 2> $O/bench_${v}_r$ring.err || { tail -5 $O/bench_${v}_r$ring.err; exit 1; }
  done
done
for f in $O/bench_*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['ms_per_step'],r['kernels_ms'],r.get('kernels_back_to_back_ms'))"; done
