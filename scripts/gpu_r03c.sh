#!/bin/bash
# Round 3: GPU test suite, smoke, the driver's exact bench command twice and a 200-step line.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03c
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYK:-} > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
for r in a b; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_$r.json 2> $OUT/bench_s20_$r.err || exit $?
done
timeout -k 10 120 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_s200.json 2> $OUT/bench_s200.err || exit $?
