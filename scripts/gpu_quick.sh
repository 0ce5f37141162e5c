#!/bin/bash
# GPU box, one call: gpu parity tests → bench (value, per-kernel and back-to-back times) → stamps of
# the given diagnostic builds.  Each GPU step has its own time limit; stop at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/bench_quick.json 2>gpurun_out/bench_quick.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_quick.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernels_ms'],r['kernels_back_to_back_ms'])"
[ $# -gt 0 ] && bash scripts/gpu_stamps_sweep.sh "$@"
exit 0
