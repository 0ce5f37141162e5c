#!/bin/bash
# Round 3: prologue L2 warm-up A/B (CVAE_WARM=1: E0's fragments; 2: + the last decoder layer's Wf/Wb)
set -u
O=gpurun_out/warm; mkdir -p $O
RING=1 CVAE_LIB=$PWD/build/diag/stw1.so timeout -k 10 90 python3 scripts/diag_stamps.py > $O/stamps_warm1.txt 2>&1 || { tail $O/stamps_warm1.txt; exit 1; }
head -8 $O/stamps_warm1.txt
VARIANTS="warm1 warm2" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
