#!/bin/bash
# Round 3: fp32-row ring chain, peer-exchange train loop, full GPU suite.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03f
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -q -k "ring_chain" --timeout 200 --timeout-method thread > $OUT/pytest_ring.log 2>&1 || { tail -40 $OUT/pytest_ring.log; exit 1; }
tail -2 $OUT/pytest_ring.log
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_peer.py -m gpu -x -v -s --timeout 400 --timeout-method thread > $OUT/pytest_peer.log 2>&1 || { tail -40 $OUT/pytest_peer.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/pytest_peer.log | tail -8
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
