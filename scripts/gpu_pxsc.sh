#!/bin/bash
# peer exchange without per-block cache maintenance (CVAE_PX_SC=1, default) vs the fenced form
# (build/diag/pxold.so): the peer parity tests, then the 2-rank rehearsal bench (both on GPU 0)
set -u
O=${O:-gpurun_out/pxsc}; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_peer.py -m gpu -q --timeout 280 --timeout-method thread > $O/tests.log 2>&1; tail -1 $O/tests.log
grep -q failed $O/tests.log && exit 1
R="timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
for i in 1 2; do
  CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 $R --master-port 2957$i bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline > $O/new_$i.json 2> $O/new_$i.err || { tail -5 $O/new_$i.err; exit 1; }
  CVAE_LIB=$PWD/build/diag/pxold.so CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 $R --master-port 2958$i bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline > $O/old_$i.json 2> $O/old_$i.err || { tail -5 $O/old_$i.err; exit 1; }
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'],d['roofline'].get('kernels_ms'),d.get('exchange_waits_rank0'))"; done
