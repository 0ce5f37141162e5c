#!/bin/bash
# GPU box, one call: parity tests → smoke → bench of library variants → in-kernel stamp diagnostics.
# Every GPU step has its own time limit; stop at the first crash/timeout (exit 124/134/137/139).
# usage: VARIANTS="default head" STAMPS=1 SUB=1 bash scripts/gpu_check.sh
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
fatal $rc && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
fatal $rc && exit $rc
for v in ${VARIANTS:-default}; do
  lib=""; [ "$v" != default ] && lib=$PWD/build/diag/$v.so
  CVAE_LIB=$lib timeout -k 10 150 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/bench_$v.json 2>gpurun_out/bench_$v.err
  rc=$?; echo "bench $v rc=$rc"; fatal $rc && exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernels_ms'])"
done
if [ "${STAMPS:-0}" = 1 ]; then
  CVAE_LIB=$PWD/build/diag/stamps.so timeout -k 10 150 python scripts/diag_stamps.py > gpurun_out/stamps.log 2>&1
  rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log | tail -40; fatal $rc && exit $rc
fi
if [ "${SUB:-0}" = 1 ]; then
  CVAE_LIB=$PWD/build/diag/sub.so timeout -k 10 150 python scripts/diag_sub.py > gpurun_out/sub.log 2>&1
  rc=$?; echo "sub rc=$rc"; grep -v amdgpu.ids gpurun_out/sub.log | tail -24; fatal $rc && exit $rc
fi
if [ "${FULLBENCH:-1}" = 1 ]; then
  timeout -k 10 200 python bench.py > gpurun_out/bench_full.json 2>gpurun_out/bench_full.err
  rc=$?; echo "full bench rc=$rc"; tail -1 gpurun_out/bench_full.json
fi
exit 0
