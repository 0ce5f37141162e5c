#!/bin/bash
# round 5: the e4m3 twin transposes converted bytes (img8), against the previous library; plus the
# timed region's fixed cost with polling signal waits (HSA_ENABLE_INTERRUPT=0) at the driver's 20 steps
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05u}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fp8 or wide or repeatable" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 scripts/repeat_check.py --workload wide --dtype fp8 --calls 300 > $O/repeat.jsonl 2>> $O/repeat.err || { cat $O/repeat.jsonl; exit 1; }
cat $O/repeat.jsonl
W="timeout -k 10 180 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-b2b --workload wide --dtype fp8"
for r in 1 2 3; do
  $W > $O/wfp8_new_$r.json 2> $O/wfp8_new_$r.err &&
  CVAE_LIB=$GRAFT_REPO_ROOT/build/ab/old.so $W > $O/wfp8_old_$r.json 2> $O/wfp8_old_$r.err || exit 1
done
B="timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-b2b"
for r in 1 2 3; do
  $B > $O/s20_def_$r.json 2> $O/s20_def_$r.err &&
  HSA_ENABLE_INTERRUPT=0 $B > $O/s20_poll_$r.json 2> $O/s20_poll_$r.err || exit 1
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
