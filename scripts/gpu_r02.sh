#!/bin/bash
# Round-2 GPU pass: pytest -m gpu, then the bench variants (each step bounded; stop at the first failure).
# usage: TAG=r02a bash scripts/gpu_r02.sh [tests|bench|all]
set -o pipefail
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
WHAT=${1:-all}
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  B="timeout -k 10 180 python -u bench.py"
  $B --steps 200 --warmup 20 > $OUT/bench_default.json 2> $OUT/bench_default.err && \
  $B --steps 200 --warmup 20 --no-cpu-baseline --dp --no-graph > $OUT/bench_dp_eager.json 2> $OUT/bench_dp_eager.err && \
  $B --steps 200 --warmup 20 --no-cpu-baseline --dp > $OUT/bench_dp_graph.json 2> $OUT/bench_dp_graph.err && \
  $B --steps 200 --warmup 20 --no-cpu-baseline --dp --graph-steps 8 > $OUT/bench_dp_graph8.json 2> $OUT/bench_dp_graph8.err && \
  $B --steps 200 --warmup 24 --no-cpu-baseline --dp --buckets 2 > $OUT/bench_dp_graph_b2.json 2> $OUT/bench_dp_graph_b2.err && \
  $B --steps 400 --warmup 20 --workload cfg1 > $OUT/bench_cfg1.json 2> $OUT/bench_cfg1.err && \
  $B --steps 400 --warmup 20 --workload cfg1 --dtype bf16 --no-cpu-baseline > $OUT/bench_cfg1_bf16.json 2> $OUT/bench_cfg1_bf16.err && \
  $B --steps 50 --warmup 5 --workload wide --no-cpu-baseline --no-b2b > $OUT/bench_wide_bf16.json 2> $OUT/bench_wide_bf16.err && \
  $B --steps 50 --warmup 5 --workload wide --dtype fp8 --no-cpu-baseline --no-b2b > $OUT/bench_wide_fp8.json 2> $OUT/bench_wide_fp8.err || \
  { echo BENCH FAILED; tail -20 $OUT/*.err; exit 1; }
  for f in $OUT/bench_*.json; do echo "$f"; python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernels_ms'], d.get('cpu_baseline',{}).get('value'))"; done
fi
if [ "$WHAT" = stamps ]; then
  CVAE_LIB=$PWD/build/diag/stamps.so timeout -k 10 120 python -u scripts/diag_stamps.py > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
  cat $OUT/stamps.txt
fi
if [ "$WHAT" = prof ]; then
  TAG=${TAG}_cfg2 PASSES=trace,sq1,sq2,fetch,write STEPS=100 bash scripts/profile.sh && \
  TAG=${TAG}_dp BENCH_EXTRA="--dp" PASSES=trace STEPS=100 bash scripts/profile.sh || exit 1
fi
