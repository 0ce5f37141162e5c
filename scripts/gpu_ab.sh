#!/bin/bash
# GPU box: parity (default library) then bench of each library variant given (default = in-tree).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log | grep -E "passed|failed"
case $rc in 0|1) ;; *) exit $rc;; esac
for v in "$@"; do
  lib=""; [ "$v" != default ] && lib=$PWD/build/diag/$v.so
  CVAE_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/bench_$v.json 2>gpurun_out/bench_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 gpurun_out/bench_$v.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernels_ms'])"
done
