#!/bin/bash
# GPU box: ring-chain tests (cfg2 bf16 path) → bench with the ring chain and with fastchain (A/B).
set -u
mkdir -p gpurun_out/ring
export TMPDIR=/tmp
K=${K:-"ring or fast or fused or bf16 or split or philox or cfg2 or misaligned or traj20 or rccl or dp"}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ring/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/ring/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/ring/pytest.log | head -30; exit $rc; }
B="timeout -k 10 180 python -u bench.py --no-cpu-baseline"
$B --steps 400 > gpurun_out/ring/bench_ring.json 2> gpurun_out/ring/bench_ring.err &&
CVAE_RING=0 $B --steps 400 > gpurun_out/ring/bench_fast.json 2> gpurun_out/ring/bench_fast.err || { tail -5 gpurun_out/ring/*.err; exit 1; }
for f in gpurun_out/ring/bench_*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernels_ms'],r.get('kernels_back_to_back_ms'))"; done
