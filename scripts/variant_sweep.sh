#!/bin/bash
# GPU box: parity (pytest -m gpu) and bench of library variants.
# usage: bash scripts/variant_sweep.sh default w4 ...   (non-default = build/diag/<name>.so)
mkdir -p gpurun_out
for v in "$@"; do
  lib=""; [ "$v" != default ] && lib=build/diag/$v.so
  CVAE_LIB=$lib timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc: $(tail -1 gpurun_out/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in "$@"; do
  lib=""; [ "$v" != default ] && lib=build/diag/$v.so
  CVAE_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/bench_$v.json 2>gpurun_out/bench_$v.err
  rc=$?; echo "$v bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernels_ms'])"
done
