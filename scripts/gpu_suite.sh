#!/bin/bash
# The whole -m gpu suite + smoke + the driver's exact bench command (round-3 tree checks).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-suite}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err || { tail -5 $OUT/bench_s20.err; exit 1; }
timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 > $OUT/bench_s200.json 2> $OUT/bench_s200.err || { tail -5 $OUT/bench_s200.err; exit 1; }
for f in $OUT/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'),r['frac'])"; done
