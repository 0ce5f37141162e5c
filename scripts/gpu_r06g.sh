#!/bin/bash
# Round 6: the -m gpu suite after the pinned non-blocking uploads, the pipelined host draws and the
# cfg4 dW decode; bench --workload cfg1 three times (the previous tree: profiles/r06f/cfg1_dec_*.json);
# an alternating A/B of bench --workload cfg4 against its tile-list dW (CVAE_CLS_DW=generic).
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06g}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for i in 1 2 3; do
  timeout -k 10 180 python3 bench.py --workload cfg1 --steps 400 --warmup 20 --no-cpu-baseline --no-b2b > $O/cfg1_$i.json 2> $O/cfg1_$i.err || exit 1
done
timeout -k 10 180 python3 bench.py --workload cfg1 > $O/cfg1_default.json 2> $O/cfg1_default.err || exit 1
B="timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --workload cfg4 --steps 200 --warmup 20"
for i in 1 2; do
  $B > $O/cfg4_dec_$i.json 2> $O/cfg4_dec_$i.err && CVAE_CLS_DW=generic $B > $O/cfg4_gen_$i.json 2> $O/cfg4_gen_$i.err || exit 1
done
for f in $O/cfg*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'),d.get('cpu_baseline',{}).get('value'))"; done
