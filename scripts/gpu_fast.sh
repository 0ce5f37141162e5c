#!/bin/bash
# GPU box: parity with the fast chain and with the generic interpreter, bench both, stamps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log | grep -E "passed|failed|Error|assert|FAIL" | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
CVAE_GENERIC=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bf16 or cfg2" > gpurun_out/pytest_gpu_generic.log 2>&1
rc=$?; echo "pytest generic rc=$rc"; tail -15 gpurun_out/pytest_gpu_generic.log | grep -E "passed|failed|Error|assert|FAIL" | head -12
case $rc in 0|1) ;; *) exit $rc;; esac
for v in fast generic; do
  g=0; [ $v = generic ] && g=1
  CVAE_GENERIC=$g timeout -k 10 150 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/bench_$v.json 2>gpurun_out/bench_$v.err
  rc=$?; echo "bench $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$v.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernels_ms'])"
done
CVAE_LIB=$PWD/build/diag/stamps.so timeout -k 10 150 python scripts/diag_stamps.py > gpurun_out/stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log | head -30
