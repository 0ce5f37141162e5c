#!/bin/bash
# GPU box: ring-chain depth sweep (build/diag/p*.so) + per-step stamps of the ring and fast chains.
set -u
O=gpurun_out/rsweep; mkdir -p $O
export TMPDIR=/tmp
B="timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 400"
for v in ${VARIANTS:-p16 p20 p24}; do
  CVAE_LIB=$PWD/build/diag/$v.so $B > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
done
$B > $O/bench_p12.json 2> $O/bench_p12.err || exit 1
for f in $O/bench_*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernels_ms'],r.get('kernels_back_to_back_ms'))"; done
RING=1 CVAE_LIB=$PWD/build/diag/rstamps.so timeout -k 10 60 python scripts/diag_stamps.py > $O/ring_stamps.txt 2>&1 || { tail $O/ring_stamps.txt; exit 1; }
CVAE_RING=0 CVAE_LIB=$PWD/build/diag/rstamps.so timeout -k 10 60 python scripts/diag_stamps.py > $O/fast_stamps.txt 2>&1 || { tail $O/fast_stamps.txt; exit 1; }
cat $O/ring_stamps.txt $O/fast_stamps.txt
