#!/bin/bash
set -u
O=gpurun_out/rep; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "repeatable" > $O/buf_$i.log 2>&1; tail -1 $O/buf_$i.log
  CVAE_LIB=$PWD/build/diag/gld.so timeout -k 10 200 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "repeatable" > $O/gld_$i.log 2>&1; tail -1 $O/gld_$i.log
done
