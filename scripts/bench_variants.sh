#!/bin/bash
# GPU box: bench only (no parity) of library variants — for diagnostic builds whose results are wrong.
mkdir -p gpurun_out
for v in "$@"; do
  lib=""; [ "$v" != default ] && lib=$PWD/build/diag/$v.so
  CVAE_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps ${STEPS:-300} ${BENCH_ARGS:-} > gpurun_out/bench_$v.json 2>gpurun_out/bench_$v.err
  rc=$?; echo "$v bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['value'],d['ms_per_step'],r['kernels_ms'],r.get('kernels_back_to_back_ms'))" gpurun_out/bench_$v.json $v
done
