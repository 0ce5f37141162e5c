#!/bin/bash
set -u
TAG=suite4 bash scripts/gpu_suite.sh || exit 1
O=gpurun_out/wst; mkdir -p $O
for dt in bf16 fp8; do
  WIDE=1 DT=$dt CVAE_LIB=$PWD/build/diag/stamps.so timeout -k 10 90 python3 scripts/diag_stamps.py > $O/wide_$dt.txt 2>&1 || { tail $O/wide_$dt.txt; exit 1; }
  tail -6 $O/wide_$dt.txt
done
