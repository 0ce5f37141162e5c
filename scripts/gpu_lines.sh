#!/bin/bash
# final-tree lines: -m gpu suite + smoke, the driver's command, cfg1 / cfg4 / cfg5 (bf16, fp8) lines (TAG)
set -u
cd $GRAFT_REPO_ROOT
T=${TAG:-lines}
O=gpurun_out/$T; mkdir -p $O
TAG=$T bash scripts/gpu_suite.sh || exit 1
timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err || exit 1
timeout -k 10 180 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_s200.json 2> $O/bench_s200.err || exit 1
timeout -k 10 180 python3 bench.py --workload cfg1 > $O/bench_cfg1.json 2> $O/bench_cfg1.err || exit 1
timeout -k 10 180 python3 bench.py --workload cfg4 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit 1
timeout -k 10 180 python3 bench.py --workload wide --no-cpu-baseline > $O/bench_wide_bf16.json 2> $O/bench_wide_bf16.err || exit 1
timeout -k 10 180 python3 bench.py --workload wide --dtype fp8 --no-cpu-baseline > $O/bench_wide_fp8.json 2> $O/bench_wide_fp8.err || exit 1
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
