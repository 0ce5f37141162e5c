#!/bin/bash
# round 5: the e4m3 wide chain's weight fragments as buffer loads (CVAE_F8_BUFLOAD=1, build/ab/bufpad.so)
# against scalar-base global loads: repeatability and parity first, then alternating bench lines
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05h}; mkdir -p $O
CVAE_LIB=$GRAFT_REPO_ROOT/build/ab/bufpad.so timeout -k 10 600 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "fp8" > $O/pytest_buf.log 2>&1 || { tail -40 $O/pytest_buf.log; exit 1; }
tail -1 $O/pytest_buf.log
for r in 1 2 3; do
  CVAE_LIB=$GRAFT_REPO_ROOT/build/ab/bufpad.so CVAE_LIB_ASSERT=0 timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/buf_$r.json 2> $O/buf_$r.err &&
  timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/glb_$r.json 2> $O/glb_$r.err || { tail -5 $O/*.err; exit 1; }
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
