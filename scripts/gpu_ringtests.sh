#!/bin/bash
set -u
O=gpurun_out/ringtests; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_hip_parity.py tests/test_gpu_cfg4.py -m gpu -q --timeout 120 --timeout-method thread -k "ring or fp32_rows or cfg2_shape" > $O/cur.log 2>&1; tail -3 $O/cur.log
grep -E "^FAILED" $O/cur.log | head
