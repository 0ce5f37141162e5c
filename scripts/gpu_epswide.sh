#!/bin/bash
# Round 3: cfg5 (wide latent) eps draws moved from the E0 GEMM into the prologue (pw2: 2 of 4, pw4: all)
set -u
O=gpurun_out/epswide; mkdir -p $O
WIDE=1 DT=bf16 VARIANTS="pw2 pw4" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab_bf16.txt 2>&1 || { tail -5 $O/ab_bf16.txt; exit 1; }
cat $O/ab_bf16.txt
WIDE=1 DT=fp8 VARIANTS="pw2 pw4" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab_fp8.txt 2>&1 || { tail -5 $O/ab_fp8.txt; exit 1; }
cat $O/ab_fp8.txt
