#!/bin/bash
# Round 3: ring fragment loads as buffer loads (default) vs 64-bit global addresses (gld), the
# Adam-scalar precompute skipped (noadam, timing only); per-block stamps of the default
set -u
O=gpurun_out/ringbuf; mkdir -p $O
RING=1 CVAE_LIB=$PWD/build/diag/stbuf.so timeout -k 10 90 python3 scripts/diag_stamps.py > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
head -25 $O/stamps.txt
VARIANTS="gld noadam" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
