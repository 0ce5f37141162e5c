#!/bin/bash
# Round 6 profiles on one MI355X: rocprofv3 kernel trace + SQ instruction mix + HBM traffic passes of
# the cfg1 fp32 chain and the cfg5 fp8 wide chain (scripts/profile.sh), then an alternating eager /
# hipGraph A/B of the cfg5 fp8 fused step.  Stops at the first failure.
set -u
cd $GRAFT_REPO_ROOT
TAG=r06_cfg1 STEPS=200 BENCH_EXTRA="--workload cfg1" PASSES=${PASSES:-trace,sq2,fetch,write} bash scripts/profile.sh || exit 1
TAG=r06_wfp8 BENCH_EXTRA="--workload wide --dtype fp8" PASSES=${PASSES:-trace,sq2,fetch,write} bash scripts/profile.sh || exit 1
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d; mkdir -p $O
B="timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 100 --warmup 10 --workload wide --dtype fp8"
for i in 1 2; do
  $B > $O/wfp8_eager_$i.json 2> $O/wfp8_eager_$i.err && $B --graph > $O/wfp8_graph_$i.json 2> $O/wfp8_graph_$i.err || exit 1
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
