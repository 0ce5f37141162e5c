#!/bin/bash
# round 5: the fp8 wide chain's new default (buffer loads + 16-state MFMA pad): fp8/wide parity and
# repeatability tests, the repeatability stress for every chain, and alternating bench lines against
# the previous default (global loads, no pad: build/ab/glb.so)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05j}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "fp8 or wide or repeatable" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R="timeout -k 10 200 python3 scripts/repeat_check.py --calls 300"
$R --workload wide --dtype fp8 --batch 1024 >> $O/repeat.jsonl 2>> $O/repeat.err &&
$R --workload wide --dtype fp8 --batch 64 >> $O/repeat.jsonl 2>> $O/repeat.err &&
$R --workload wide --dtype bf16 --batch 1024 >> $O/repeat.jsonl 2>> $O/repeat.err &&
$R --workload cfg2 --dtype bf16 --batch 1024 >> $O/repeat.jsonl 2>> $O/repeat.err || { cat $O/repeat.jsonl; tail -5 $O/repeat.err; exit 1; }
cat $O/repeat.jsonl
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 --workload wide --dtype fp8"
for r in 1 2 3; do
  $B > $O/new_$r.json 2> $O/new_$r.err &&
  CVAE_LIB=$GRAFT_REPO_ROOT/build/ab/glb.so $B > $O/old_$r.json 2> $O/old_$r.err || { tail -5 $O/*.err; exit 1; }
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
