#!/bin/bash
# post-change check: the driver's bench command, the 2-rank rehearsal (peer exchange self-check) and
# the peer tests, each under its own limit; stops at the first failure
set -u
O=${O:-gpurun_out/chk}; mkdir -p $O
timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err || { tail -5 $O/bench_s20.err; exit 1; }
CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_share2.json 2> $O/bench_share2.err || { tail -5 $O/bench_share2.err; exit 1; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_peer.py -m gpu -q --timeout 280 --timeout-method thread > $O/peer_tests.log 2>&1 || { tail -20 $O/peer_tests.log; exit 1; }
tail -1 $O/peer_tests.log
for f in $O/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d.get('exchange_verified'))"; done
