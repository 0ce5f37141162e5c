#!/bin/bash
# Round 3: per-block stamps (is block 0, which precomputes the Adam scalars, the slowest?) + A/B
set -u
O=gpurun_out/adampre; mkdir -p $O
RING=1 CVAE_LIB=$PWD/build/diag/stamps.so timeout -k 10 90 python3 scripts/diag_stamps.py > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
head -24 $O/stamps.txt
VARIANTS="noadam" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
