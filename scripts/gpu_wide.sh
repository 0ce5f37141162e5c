#!/bin/bash
# GPU box: the cfg5 wide-chain tests, then the whole GPU suite, then the wide bench (bf16).
# Each GPU step has its own time limit; stop at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "wide or fp8" > gpurun_out/pytest_wide.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_wide.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload wide --no-cpu-baseline --steps 100 > gpurun_out/bench_wide.json 2>gpurun_out/bench_wide.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_wide.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_wide.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernels_ms'],r.get('kernels_back_to_back_ms'))"
exit 0
