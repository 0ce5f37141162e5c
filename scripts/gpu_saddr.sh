#!/bin/bash
# Round 3: the e4m3 wide chain's fragment loads with a scalar base + 32-bit lane offset (saddr)
# vs 64-bit per-lane addresses: repeatability tests, then the cfg5 fp8 bench A/B
set -u
O=gpurun_out/saddr; mkdir -p $O
for i in 1 2; do
  CVAE_LIB=$PWD/build/diag/saddr.so timeout -k 10 200 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "repeatable or wide" > $O/saddr_$i.log 2>&1; tail -1 $O/saddr_$i.log
done
grep -q failed $O/saddr_1.log $O/saddr_2.log && exit 1
WIDE=1 DT=fp8 VARIANTS="saddr" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
RING=1 SUB=1 CVAE_LIB=$PWD/build/diag/sub2.so timeout -k 10 90 python3 scripts/diag_stamps.py > $O/sub2.txt 2>&1 || { tail $O/sub2.txt; exit 1; }
head -30 $O/sub2.txt
