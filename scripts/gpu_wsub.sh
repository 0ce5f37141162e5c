#!/bin/bash
set -u
O=gpurun_out/wst; mkdir -p $O
for dt in bf16 fp8; do
  SUB=1 WIDE=1 DT=$dt CVAE_LIB=$PWD/build/diag/wsub.so timeout -k 10 90 python scripts/diag_stamps.py > $O/wsub_$dt.txt 2>&1 || { tail $O/wsub_$dt.txt; exit 1; }
done
paste $O/wsub_bf16.txt $O/wsub_fp8.txt | cut -c1-160 | head -16
