#!/bin/bash
# GPU box: B_local sweep of the training step (SURVEY §8d "MFMA utilisation ... with a B_local
# sweep {1024, 4096, 16384, 65536}"): bench.py per batch, then one rocprofv3 PMC pass per batch
# with the MFMA-busy and clock counters.  Writes gpurun_out/bsweep/; stops at the first failure.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/bsweep
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BATCHES=${BATCHES:-"1024 4096 16384 65536"}
for B in $BATCHES; do
  STEPS=$(( 200 * 1024 / B )); [ $STEPS -lt 20 ] && STEPS=20
  timeout -k 10 240 python3 $GRAFT_REPO_ROOT/bench.py --batch $B --steps $STEPS --warmup 5 --no-cpu-baseline \
      > $OUT/bench_$B.json 2> $OUT/bench_$B.err || { tail -5 $OUT/bench_$B.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
      --output-format csv -d $OUT -o pmc_$B -- python3 $GRAFT_REPO_ROOT/bench.py --batch $B --steps 20 --warmup 2 \
      --no-cpu-baseline --no-b2b > $OUT/pmc_$B.log 2>&1 || { echo "pmc $B failed"; tail -5 $OUT/pmc_$B.log; exit 1; }
  echo "B=$B ok"
done
python3 $GRAFT_REPO_ROOT/scripts/bsweep_summary.py $OUT > $OUT/summary.md && cat $OUT/summary.md
