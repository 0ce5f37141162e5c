#!/bin/bash
# Round 3: eps draw placement A/B at cfg2 (w0: only wave 0 draws, in E0; pro: the draw in the
# prologue while the x tile loads; prow0: both)
set -u
O=gpurun_out/epsab; mkdir -p $O
RING=1 CVAE_LIB=$PWD/build/diag/stprow0.so timeout -k 10 90 python3 scripts/diag_stamps.py > $O/stamps_prow0.txt 2>&1 || { tail $O/stamps_prow0.txt; exit 1; }
head -8 $O/stamps_prow0.txt
VARIANTS="w0 pro prow0" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
