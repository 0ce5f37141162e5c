#!/bin/bash
# round 5: the shared-GPU rehearsals with one HIP hardware queue per rank (bench.py rank_envs now
# sets it in share mode; the peer tests' workers too) — the 8-rank rehearsal was 46 ms per step with
# HIP's default 4 queues per process (the GPU's queue slots oversubscribed, ranks time-sliced)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05w}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_peer.py -x -v -rP --timeout 300 --timeout-method thread > $O/pytest_peer.log 2>&1 || { tail -30 $O/pytest_peer.log; exit 1; }
tail -1 $O/pytest_peer.log; grep "owner waits" $O/pytest_peer.log | cut -c1-200
for n in 2 4 8; do
  CVAE_BENCH_SHARE_GPU=1 timeout -k 10 400 python3 bench.py --gpus $n --steps 20 --warmup 5 \
    > $O/share${n}.json 2> $O/share${n}.err || { tail -5 $O/share${n}.err; exit 1; }
done
for f in $O/share?.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'),d.get('exchange_verified'),d.get('exchange_verified_after'),d.get('exchange_waits_rank0'))"; done
