#!/bin/bash
# Round 3: per-CU stream microbenchmark (hot-channel test), then the peer tests and rehearsals.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03g
mkdir -p $OUT
timeout -k 10 120 $GRAFT_REPO_ROOT/scripts/ubench/stream > $OUT/stream.txt 2>&1 || { cat $OUT/stream.txt; exit 1; }
cat $OUT/stream.txt
bash $GRAFT_REPO_ROOT/scripts/gpu_peer.sh
