#!/bin/bash
# GPU box: bench only (no parity) of library variants — for diagnostic builds whose results are wrong.
mkdir -p gpurun_out
for v in "$@"; do
  lib=""; [ "$v" != default ] && lib=build/diag/$v.so
  CVAE_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/bench_$v.json 2>gpurun_out/bench_$v.err
  rc=$?; echo "$v bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernels_ms'])"
done
