#!/bin/bash
# GPU-box check: parity tests → smoke → bench.  Stops at the first crash/timeout
# (exit 124/134/137/139); ordinary test failures (exit 1) still let the bench run.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { case "$1" in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 ${PYTEST_T:-600} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
