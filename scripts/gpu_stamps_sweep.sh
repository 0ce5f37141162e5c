#!/bin/bash
# GPU box: per-step stamp profile (scripts/diag_stamps.py) of each diagnostic build given.
mkdir -p gpurun_out
for v in "$@"; do
  CVAE_LIB=$PWD/build/diag/$v.so timeout -k 10 120 python scripts/diag_stamps.py > gpurun_out/stamps_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -v amdgpu.ids gpurun_out/stamps_$v.log | awk '{print}' | tr -s ' ' | cut -c1-120
done
