#!/bin/bash
# round 5: the fused cfg2 step eager (one prepared C call) vs replayed from a captured hipGraph
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05e}; mkdir -p $O
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-b2b"
for r in 1 2; do
  $B --steps 200 --warmup 20 > $O/eager_$r.json 2> $O/eager_$r.err &&
  $B --steps 200 --warmup 20 --graph --graph-steps 8 > $O/graph8_$r.json 2> $O/graph8_$r.err &&
  $B --steps 200 --warmup 20 --graph --graph-steps 40 > $O/graph40_$r.json 2> $O/graph40_$r.err &&
  $B --steps 20 --warmup 5 --graph --graph-steps 20 > $O/graph20_s20_$r.json 2> $O/graph20_s20_$r.err &&
  $B --steps 20 --warmup 5 > $O/eager_s20_$r.json 2> $O/eager_s20_$r.err || { tail -5 $O/*.err; exit 1; }
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'),d['config']['workload'][-60:])"; done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dp_autograd.py -m gpu -x -v -rP --timeout 120 --timeout-method thread -k "rccl" > $O/pytest_rccl.log 2>&1 || { tail -30 $O/pytest_rccl.log; exit 1; }
tail -1 $O/pytest_rccl.log
for r in 1 2; do
  $B --steps 200 --warmup 20 --dp > $O/dp_native_$r.json 2> $O/dp_native_$r.err &&
  $B --steps 200 --warmup 20 --dp --buckets 2 > $O/dp_native_b2_$r.json 2> $O/dp_native_b2_$r.err &&
  $B --steps 200 --warmup 20 --dp --torch-allreduce > $O/dp_torch_$r.json 2> $O/dp_torch_$r.err &&
  $B --steps 200 --warmup 20 --dp --buckets 2 --torch-allreduce > $O/dp_torch_b2_$r.json 2> $O/dp_torch_b2_$r.err || { tail -5 $O/*.err; exit 1; }
done
for f in $O/dp*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
