#!/bin/bash
# round 5: run-to-run repeatability stress (300 forward_backward calls, B = 1024 and 64) of the fp8
# wide chain: the default build (scalar-base global loads), buffer loads with the 16-state pad after
# each e4m3 MFMA (build/ab/bufpad.so), buffer loads without it (build/ab/buf.so, expected to fail)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05i}; mkdir -p $O
R="timeout -k 10 200 python3 scripts/repeat_check.py --workload wide --dtype fp8 --calls 300"
for b in 1024 64; do
  $R --batch $b >> $O/repeat.jsonl 2>> $O/repeat.err; echo "default B=$b rc $?"
  CVAE_LIB=$GRAFT_REPO_ROOT/build/ab/bufpad.so $R --batch $b >> $O/repeat.jsonl 2>> $O/repeat.err; echo "bufpad B=$b rc $?"
  CVAE_LIB=$GRAFT_REPO_ROOT/build/ab/buf.so $R --batch $b >> $O/repeat.jsonl 2>> $O/repeat.err; echo "buf B=$b rc $?"
done
cat $O/repeat.jsonl
