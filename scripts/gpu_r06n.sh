#!/bin/bash
# Round 6: the next step's rows gathered in the fp32 dW launch — the fp32-chain tests, then an
# alternating A/B of bench --workload cfg1 against CVAE_GATHER_AHEAD=0.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06n}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_f32chain.py tests/test_hip_parity.py tests/test_gpu_dp_autograd.py -v -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-b2b --workload cfg1 --steps 400 --warmup 20"
for i in 1 2 3; do
  $B > $O/cfg1_ahead_$i.json 2> $O/cfg1_ahead_$i.err && CVAE_GATHER_AHEAD=0 $B > $O/cfg1_chain_$i.json 2> $O/cfg1_chain_$i.err || exit 1
done
for f in $O/cfg1_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
