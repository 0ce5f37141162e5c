#!/bin/bash
# GPU box: per-step stamps of the wide chain, bf16 and the fp8 form (build/diag/wstamps.so).
set -u
O=gpurun_out/wst; mkdir -p $O
for dt in bf16 fp8; do
  WIDE=1 DT=$dt CVAE_LIB=$PWD/build/diag/wstamps.so timeout -k 10 90 python scripts/diag_stamps.py > $O/wide_$dt.txt 2>&1 || { tail $O/wide_$dt.txt; exit 1; }
done
paste $O/wide_bf16.txt $O/wide_fp8.txt | cut -c1-160
