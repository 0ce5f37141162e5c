#!/bin/bash
# GPU box: time each diagnostic variant with bench.py (no CPU baseline).
mkdir -p gpurun_out
for v in base nowpack nostore nostore_nowpack; do
  CVAE_LIB=build/diag/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/diag_$v.json 2>gpurun_out/diag_$v.err
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/diag_$v.json'));print('$v', d['ms_per_step'], d['roofline']['kernels_ms'])"
done
