#!/bin/bash
# Round 3: the peer-exchange tests (several ranks on the box's one GPU).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/peer
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_peer.py -m gpu -v -s --timeout 300 --timeout-method thread ${PYK:-} > $OUT/pytest_peer.log 2>&1
rc=$?
grep -E "rank [0-9]: fault|PASS|FAIL|passed|failed" $OUT/pytest_peer.log | head -60
[ $rc -ne 0 ] && exit $rc
# the bench's N>1 path end to end (2 ranks sharing GPU 0, gloo for host collectives; not a scaling number)
CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_share2.json 2> $OUT/bench_share2.err
rc2=$?
cat $OUT/bench_share2.json | head -c 1500; echo
exit $rc2
