#!/bin/bash
# round 5: leaner loss-epilogue indexing + the e4m3 scale selects on wave 0 only, against the previous
# library; the e4m3 form's prologue eps draws 0 / 2 (default) / 4 — alternating bench lines
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05s}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_parity.py tests/test_gpu_cfg4.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
A=$GRAFT_REPO_ROOT/build/ab
W="timeout -k 10 180 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-b2b --workload wide --dtype fp8"
C="timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-b2b"
for r in 1 2 3; do
  for v in new old eps0 eps4; do
    L=""; [ $v != new ] && L=$A/$v.so
    CVAE_LIB=$L $W > $O/wfp8_${v}_$r.json 2> $O/wfp8_${v}_$r.err || { tail -3 $O/wfp8_${v}_$r.err; exit 1; }
  done
  for v in new old; do
    L=""; [ $v != new ] && L=$A/$v.so
    CVAE_LIB=$L $C > $O/cfg2_${v}_$r.json 2> $O/cfg2_${v}_$r.err || { tail -3 $O/cfg2_${v}_$r.err; exit 1; }
  done
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
