#!/bin/bash
# Round 3: cfg4 on the ring chain — its tests, the whole GPU suite, and a cfg4 bench line.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03e
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_cfg4.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_cfg4.log 2>&1 || { tail -40 $OUT/pytest_cfg4.log; exit 1; }
grep -E "PASS|FAIL" $OUT/pytest_cfg4.log | tail -12
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python3 bench.py --workload cfg4 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err || { tail -5 $OUT/bench_cfg4.err; exit 1; }
timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.err || exit 1
for f in $OUT/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernels_ms'])"; done
