#!/bin/bash
# Round 4, first check of the exchange hardening: the peer tests (world 2/3/4 with the residency
# bound, the resume re-arm), the bf16 reconstruction parity test, the driver's bench command and the
# 2- and 4-rank rehearsals of the N>1 path (both self-checks in the line).  Each GPU step has its
# own limit; the script stops at the first failure.
set -u
O=${O:-gpurun_out/r04a}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_peer.py tests/test_hip_parity.py -m gpu -x -v \
  -k "peer or reconstruction or cfg2_shape" --timeout 280 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|bf16 ring chain|vs bf16 emulation" $O/tests.log | tail -20
timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err || { tail -5 $O/bench_s20.err; exit 1; }
for n in 2 4; do
  CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2957$n bench.py --gpus $n --steps 20 --warmup 5 \
    > $O/bench_share$n.json 2> $O/bench_share$n.err || { tail -5 $O/bench_share$n.err; exit 1; }
done
for f in $O/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d.get('exchange_verified'),d.get('exchange_verified_after'),d.get('exchange_layout'))"; done
