#!/bin/bash
# round 5: the whole -m gpu suite on the new library (bf16-dX fallback, tap rule, occupancy-derived
# exchange slots, cfg3 peer cases), then cfg5 fp8 bench lines of both dX forms
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05b}; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline"
$B --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/wfp8_mx.json 2> $O/wfp8_mx.err &&
CVAE_FP8_DX=bf16 $B --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/wfp8_bdx.json 2> $O/wfp8_bdx.err &&
$B --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/wfp8_mx2.json 2> $O/wfp8_mx2.err &&
CVAE_FP8_DX=bf16 $B --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/wfp8_bdx2.json 2> $O/wfp8_bdx2.err || { tail -5 $O/*.err; exit 1; }
for f in $O/w*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
