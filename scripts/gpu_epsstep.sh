#!/bin/bash
# Round 3: cfg5 stepped Philox draws (step.so) — wide-chain tests with it, then the bench A/B
set -u
O=gpurun_out/epsstep; mkdir -p $O
CVAE_LIB=$PWD/build/diag/step.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "wide" > $O/tests.log 2>&1; tail -1 $O/tests.log
grep -q failed $O/tests.log && exit 1
WIDE=1 DT=bf16 VARIANTS="step" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab_bf16.txt 2>&1 || { tail -5 $O/ab_bf16.txt; exit 1; }
cat $O/ab_bf16.txt
WIDE=1 DT=fp8 VARIANTS="step" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab_fp8.txt 2>&1 || { tail -5 $O/ab_fp8.txt; exit 1; }
cat $O/ab_fp8.txt
