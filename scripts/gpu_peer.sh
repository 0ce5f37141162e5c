#!/bin/bash
# Round 3: the peer-exchange tests (several ranks on the box's one GPU) and the bench's N>1 path
# rehearsed with ranks sharing GPU 0 (gloo for the host-side collectives; not a scaling number).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/peer
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_peer.py -m gpu -v -s --timeout 400 --timeout-method thread ${PYK:-} > $OUT/pytest_peer.log 2>&1
rc=$?
grep -E "rank [0-9]: fault|PASS|FAIL|passed|failed" $OUT/pytest_peer.log | head -60
[ $rc -ne 0 ] && exit $rc
for n in 2 3; do
  CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2956$n bench.py --gpus $n --steps 20 --warmup 5 > $OUT/bench_share$n.json 2> $OUT/bench_share$n.err || { tail -5 $OUT/bench_share$n.err; exit 1; }
  head -c 700 $OUT/bench_share$n.json; echo
done
