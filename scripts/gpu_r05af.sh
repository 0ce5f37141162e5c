#!/bin/bash
# round 5: the Adam scalars' two f64 pows on two waves of block 0 (cfg2, cfg4), the step count stored
# after the prologue barrier, against the previous library (502910c)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05af}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in new old; do
    L=""; [ $v = old ] && L=$GRAFT_REPO_ROOT/build/ab/old.so
    CVAE_LIB=$L timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-b2b > $O/s20_${v}_$r.json 2> $O/s20_${v}_$r.err &&
    CVAE_LIB=$L timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-b2b > $O/s200_${v}_$r.json 2> $O/s200_${v}_$r.err &&
    CVAE_LIB=$L timeout -k 10 180 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-b2b --workload wide --dtype fp8 > $O/wfp8_${v}_$r.json 2> $O/wfp8_${v}_$r.err &&
    CVAE_LIB=$L timeout -k 10 180 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-b2b --workload wide > $O/wbf16_${v}_$r.json 2> $O/wbf16_${v}_$r.err || exit 1
  done
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
