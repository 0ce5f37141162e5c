#!/bin/bash
# the train loop over the peer exchange: current library vs build/diag/prev.so
set -u
O=gpurun_out/peerab; mkdir -p $O
T="timeout -k 10 300 python3 -u -m pytest tests/test_gpu_peer.py -m gpu -q --timeout 280 --timeout-method thread -k train_loop"
CVAE_LIB=$PWD/build/diag/prev.so $T > $O/prev.log 2>&1; tail -1 $O/prev.log
$T > $O/cur.log 2>&1; tail -1 $O/cur.log
