#!/bin/bash
# round 5: the x-tile transform as a register transpose (timestep-pair tasks, no DPP): the whole GPU
# suite, then alternating bench lines against the previous library (build/ab/old.so): cfg2 in the
# driver's 20-step form and at 200 steps, cfg5 fp8 and bf16
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05k}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
OLD=$GRAFT_REPO_ROOT/build/ab/old.so
for r in 1 2 3; do
  for v in new old; do
    L=""; [ $v = old ] && L=$OLD
    CVAE_LIB=$L timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s20_${v}_$r.json 2> $O/s20_${v}_$r.err &&
    CVAE_LIB=$L timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/s200_${v}_$r.json 2> $O/s200_${v}_$r.err &&
    CVAE_LIB=$L timeout -k 10 180 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --workload wide --dtype fp8 > $O/wfp8_${v}_$r.json 2> $O/wfp8_${v}_$r.err &&
    CVAE_LIB=$L timeout -k 10 180 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --workload wide > $O/wbf16_${v}_$r.json 2> $O/wbf16_${v}_$r.err || { tail -5 $O/*.err; exit 1; }
  done
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
