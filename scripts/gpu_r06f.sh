#!/bin/bash
# Round 6: the fp32 chain's compile-time dW decode (cvae_f32wgrad.h) — its parity tests, then an
# alternating A/B of bench --workload cfg1 against the tile-list kernel (CVAE_F32_DW=generic).
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06f}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_f32chain.py tests/test_hip_parity.py -v -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --workload cfg1 --steps 400 --warmup 20"
for i in 1 2 3; do
  $B > $O/cfg1_dec_$i.json 2> $O/cfg1_dec_$i.err && CVAE_F32_DW=generic $B > $O/cfg1_gen_$i.json 2> $O/cfg1_gen_$i.err || exit 1
done
for f in $O/cfg1_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
