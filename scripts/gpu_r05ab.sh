#!/bin/bash
# round 5: sub-stamps of the final chains (cfg2 ring, cfg5 fp8)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05ab}; mkdir -p $O
S="timeout -k 10 120 python3 scripts/diag_stamps.py"
CVAE_LIB=$PWD/build/ab/stamps2.so RING=1 SUB=1 $S > $O/substamps_cfg2.txt 2>&1 &&
CVAE_LIB=$PWD/build/ab/stamps2.so WIDE=1 SUB=1 DT=fp8 $S > $O/substamps_wide_fp8.txt 2>&1 || { tail -5 $O/*.txt; exit 1; }
sed -n 2,12p $O/substamps_cfg2.txt; sed -n 2,8p $O/substamps_wide_fp8.txt
