#!/bin/bash
# The peer exchange at world 8 rehearsed on the box's one GPU (8 rank processes): the parity test,
# then the bench's N > 1 path with 8 ranks (a rehearsal of the driver's 8-GPU command, not a
# scaling number).
set -u
O=gpurun_out/w8; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_peer.py -m gpu -x -v -s -k w8 --timeout 280 --timeout-method thread > $O/pytest_w8.log 2>&1 || { tail -30 $O/pytest_w8.log; exit 1; }
grep -E "rank [0-9]: fault|passed|failed" $O/pytest_w8.log | cut -c1-200
CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29588 bench.py --gpus 8 --steps 20 --warmup 5 \
  > $O/bench_share8.json 2> $O/bench_share8.err || { tail -20 $O/bench_share8.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_share8.json'));print(d['value'],d['ms_per_step'],d['config'].get('workload'),d.get('exchange_verified'),d.get('exchange_verified_after'),d['roofline'].get('kernels_ms'))"
