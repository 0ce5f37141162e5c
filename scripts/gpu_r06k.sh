#!/bin/bash
# Round 6: the eps drawn ahead — its bit-equality tests, then an alternating A/B of the wide benches
# against every chain drawing its own (CVAE_EPS_AHEAD=0).
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06k}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_eps_ahead.py -v -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 100 --warmup 10 --workload wide"
for i in 1 2; do
  $B --dtype fp8 > $O/wfp8_ahead_$i.json 2> $O/wfp8_ahead_$i.err && CVAE_EPS_AHEAD=0 $B --dtype fp8 > $O/wfp8_chain_$i.json 2> $O/wfp8_chain_$i.err || exit 1
  $B > $O/wbf16_ahead_$i.json 2> $O/wbf16_ahead_$i.err && CVAE_EPS_AHEAD=0 $B > $O/wbf16_chain_$i.json 2> $O/wbf16_chain_$i.err || exit 1
done
for f in $O/w*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
