#!/bin/bash
# Round 3: cfg2 prologue A/B — ring fill split around the x-tile wait (pf4: 4 items before, pf0: none
# before) and the per-row start point by 8-B loads (x08)
set -u
O=gpurun_out/prologue; mkdir -p $O
VARIANTS="pf4 pf0 x08" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
