#!/bin/bash
# GPU box: full GPU suite, then the data-parallel step structure at one rank (dp_overhead) with its kernel trace.
set -u
mkdir -p gpurun_out/dp; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_dp_prof.sh
