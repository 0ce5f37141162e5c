set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 60 scripts/ubench/phase D > $O/phase_d.txt 2>&1 || { cat $O/phase_d.txt; exit 1; }
cat $O/phase_d.txt
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_peer.py -x -v -rP --timeout 600 --timeout-method thread -k "cfg3 or w8" > $O/peer.log 2>&1 || { tail -30 $O/peer.log; exit 1; }
tail -3 $O/peer.log
CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $O/share2.json 2> $O/share2.err || { echo rc $?; tail -20 $O/share2.err; exit 1; }
cat $O/share2.json
CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 timeout -k 10 400 python3 bench.py --gpus 8 --steps 20 --warmup 5 > $O/share8.json 2> $O/share8.err || { echo rc $?; tail -20 $O/share8.err; exit 1; }
cat $O/share8.json
timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/s20.json 2> $O/s20.err || exit 1
cat $O/s20.json
