#!/bin/bash
# split-K hand-off in the sc1 form: split-K tests, then the B_local sweep
set -u
O=gpurun_out/splitk; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "splitk" > $O/tests.log 2>&1; tail -1 $O/tests.log
grep -q failed $O/tests.log && exit 1
bash scripts/bsweep.sh
