#!/bin/bash
# round 5: the fp8 wide chain after the VALU cuts (one-instruction e4m3 saturation, the KL sum in the
# decoder-L0 backward) and the MX dW (CVAE_FP8_DW=mx): its parity tests, then alternating bench lines
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05c}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "fp8 or wide" > $O/pytest_fp8.log 2>&1 || { tail -40 $O/pytest_fp8.log; exit 1; }
tail -2 $O/pytest_fp8.log
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 --workload wide"
for r in 1 2; do
  $B --dtype fp8 > $O/wfp8_$r.json 2> $O/wfp8_$r.err &&
  CVAE_FP8_DW=mx $B --dtype fp8 > $O/wfp8_mxdw_$r.json 2> $O/wfp8_mxdw_$r.err &&
  $B > $O/wbf16_$r.json 2> $O/wbf16_$r.err || { tail -5 $O/*.err; exit 1; }
done
timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 > $O/cfg2.json 2> $O/cfg2.err || exit 1
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
