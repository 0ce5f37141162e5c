#!/bin/bash
# Round 3: price the last decoder layer's loss epilogue (noloss: timing only)
set -u
O=gpurun_out/lossepi; mkdir -p $O
for v in stamps stnoloss; do
  RING=1 CVAE_LIB=$PWD/build/diag/$v.so timeout -k 10 90 python3 scripts/diag_stamps.py > $O/$v.txt 2>&1 || { tail $O/$v.txt; exit 1; }
done
paste $O/stamps.txt $O/stnoloss.txt | cut -c1-210 | head -24
VARIANTS="noloss" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
