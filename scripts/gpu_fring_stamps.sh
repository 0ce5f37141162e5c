#!/bin/bash
# Round 3: in-kernel stamps of the two-launch ring step and the one-launch step (build/diag/stamps.so).
set -u
O=gpurun_out/frst; mkdir -p $O
for v in 0 1; do
  CVAE_FUSE_RING=$v RING=1 CVAE_LIB=$PWD/build/diag/stamps.so timeout -k 10 90 python3 scripts/diag_stamps.py > $O/fring$v.txt 2>&1 || { tail $O/fring$v.txt; exit 1; }
  cat $O/fring$v.txt
done
