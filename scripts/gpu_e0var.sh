#!/bin/bash
# encoder-L1 GEMM variants (row tiles per wave _ waves per workgroup _ chunks prefetched), M = 2^20
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/e0gemm
mkdir -p $OUT
for v in 4_8_3 4_8_4 2_16_3 2_16_4; do
  timeout -k 10 60 $GRAFT_REPO_ROOT/scripts/ubench/e0gemm_$v 1048576 50 > $OUT/var_$v.json 2>&1 || { cat $OUT/var_$v.json; exit 1; }
  echo "$v $(cat $OUT/var_$v.json)"
done
