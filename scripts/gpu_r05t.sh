#!/bin/bash
# round 5: the timed region's fixed cost (first launch + final synchronise) at the driver's 20 steps:
# default signal waits against polling ones (HSA_ENABLE_INTERRUPT=0), alternating
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05t}; mkdir -p $O
B="timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-b2b"
for r in 1 2 3; do
  $B > $O/def_$r.json 2> $O/def_$r.err || exit 1
  HSA_ENABLE_INTERRUPT=0 $B > $O/poll_$r.json 2> $O/poll_$r.err || exit 1
done
HSA_ENABLE_INTERRUPT=0 timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-b2b > $O/poll_s200.json 2> $O/poll_s200.err || exit 1
timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-b2b > $O/def_s200.json 2> $O/def_s200.err || exit 1
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
