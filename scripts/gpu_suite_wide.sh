#!/bin/bash
# GPU suite + smoke + driver command + 200 steps, then the cfg5 wide lines (bf16, fp8)
set -u
TAG=${TAG:-suite6} bash scripts/gpu_suite.sh || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-suite6}
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline"
for i in 1 2; do
  $B --steps 100 --warmup 10 --workload wide > $OUT/wide_bf16_$i.json 2> $OUT/wide_bf16_$i.err || { tail -3 $OUT/wide_bf16_$i.err; exit 1; }
  $B --steps 100 --warmup 10 --workload wide --dtype fp8 > $OUT/wide_fp8_$i.json 2> $OUT/wide_fp8_$i.err || { tail -3 $OUT/wide_fp8_$i.err; exit 1; }
done
for f in $OUT/wide_*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
