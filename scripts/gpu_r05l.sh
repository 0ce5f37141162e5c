#!/bin/bash
# round 5: sub-stamps of the three chains after the transform change (diagnostic build)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05l}; mkdir -p $O
S="timeout -k 10 120 python3 scripts/diag_stamps.py"
CVAE_LIB=$PWD/build/ab/stamps2.so WIDE=1 SUB=1 DT=fp8 $S > $O/substamps_wide_fp8.txt 2>&1 &&
CVAE_LIB=$PWD/build/ab/stamps2.so WIDE=1 SUB=1 DT=bf16 $S > $O/substamps_wide_bf16.txt 2>&1 &&
CVAE_LIB=$PWD/build/ab/stamps2.so RING=1 SUB=1 $S > $O/substamps_cfg2.txt 2>&1 || { tail -5 $O/*.txt; exit 1; }
head -60 $O/substamps_wide_fp8.txt | grep -v "^  " ; head -40 $O/substamps_cfg2.txt | grep -v "^  "
