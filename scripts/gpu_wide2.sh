#!/bin/bash
# GPU box: wide-chain tests → wide bench (default + variants given as args) → wide stamps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wide or fp8" > gpurun_out/pytest_wide.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_wide.log; [ $rc -eq 0 ] || exit $rc
STEPS=100 BENCH_ARGS="--workload wide" bash scripts/bench_variants.sh default "$@" || exit $?
WIDE=1 CVAE_LIB=$PWD/build/diag/wstamps.so timeout -k 10 60 python scripts/diag_stamps.py > gpurun_out/wstamps.txt 2>&1
rc=$?; cat gpurun_out/wstamps.txt; exit $rc
