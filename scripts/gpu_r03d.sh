#!/bin/bash
# Round 3: dW-kernel A/B (one-wave decode, write-through epilogue stores) + the GPU suite.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03d
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
VARIANTS="olddw dec0 wt0" timeout -k 10 600 bash scripts/gpu_variant_ab.sh > $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
cp -r gpurun_out/vab $OUT/
cat $OUT/ab.txt
