#!/bin/bash
# round 5: cfg5's dW ⊕ Adam on 64 x 64 tiles (widewgrad64_kernel) against the 32 x 64 tiles (CVAE_DW64=0)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05f}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "wide" > $O/pytest_wide.log 2>&1 || { tail -40 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 --workload wide"
for r in 1 2; do
  $B --dtype fp8 > $O/wfp8_64_$r.json 2> $O/wfp8_64_$r.err &&
  CVAE_DW64=0 $B --dtype fp8 > $O/wfp8_32_$r.json 2> $O/wfp8_32_$r.err &&
  $B > $O/wbf16_64_$r.json 2> $O/wbf16_64_$r.err &&
  CVAE_DW64=0 $B > $O/wbf16_32_$r.json 2> $O/wbf16_32_$r.err || { tail -5 $O/*.err; exit 1; }
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
for r in 1 2; do
  CVAE_LIB=$GRAFT_REPO_ROOT/build/ab/pf4.so $B --dtype fp8 > $O/wfp8_64pf4_$r.json 2> $O/wfp8_64pf4_$r.err &&
  $B --dtype fp8 > $O/wfp8_64b_$r.json 2> $O/wfp8_64b_$r.err || { tail -5 $O/*.err; exit 1; }
done
for f in $O/wfp8_64*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
