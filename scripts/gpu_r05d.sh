#!/bin/bash
# round 5: the fp8 wide chain with the x_rel e4m3 twin written by the prologue transform
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05d}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "fp8 or wide" > $O/pytest_fp8.log 2>&1 || { tail -40 $O/pytest_fp8.log; exit 1; }
tail -1 $O/pytest_fp8.log
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 --workload wide --dtype fp8"
for r in 1 2 3; do $B > $O/wfp8_$r.json 2> $O/wfp8_$r.err || { tail -5 $O/wfp8_$r.err; exit 1; }; done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
