#!/bin/bash
# Round 3, Next #1: the driver's exact bench command, its rocprofv3 kernel trace, a 200-step line
# beside it, and the short-run decomposition (scripts/short_run.py).  Stops at the first failure.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03a
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_a.json 2> $OUT/bench_s20_a.err || exit $?
timeout -k 10 120 python3 bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/bench_s200.json 2> $OUT/bench_s200.err || exit $?
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_b.json 2> $OUT/bench_s20_b.err || exit $?
timeout -k 10 180 python3 scripts/short_run.py > $OUT/short_run.json 2> $OUT/short_run.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o s20 -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_s20.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o s200 -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/prof_s200.log 2>&1 || exit $?
find $OUT -name '*.csv' | head -20
