#!/bin/bash
# Round 3: short-run fixed cost — eager vs prepared call vs captured K-step graph (scripts/short_run.py)
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03b
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for m in prepared graph eager; do
  timeout -k 10 180 python3 scripts/short_run.py $m > $OUT/short_$m.json 2> $OUT/short_$m.err || exit $?
done
