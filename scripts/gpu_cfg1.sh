#!/bin/bash
# the -m gpu suite + smoke, the driver's command, cfg1 bench lines, its kernel trace and
# PMC / traffic passes (TAG=...)
set -u
cd $GRAFT_REPO_ROOT
T=${TAG:-cfg1}
O=gpurun_out/$T; mkdir -p $O
TAG=$T bash scripts/gpu_suite.sh || exit 1
timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err || exit 1
timeout -k 10 180 python3 bench.py --workload cfg1 > $O/bench_cfg1.json 2> $O/bench_cfg1.err || exit 1
timeout -k 10 180 python3 bench.py --workload cfg1 --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_cfg1_400.json 2> $O/bench_cfg1_400.err || exit 1
TAG=${T}_cfg1 PASSES=trace,sq2,tcc,fetch,write STEPS=200 BENCH_EXTRA="--workload cfg1" bash scripts/profile.sh || exit 1
python3 scripts/pmc_traffic.py gpurun_out/prof ${T}_cfg1 gpurun_out/prof/${T}_cfg1_traffic.json 32 fp32 > /dev/null &&
python3 scripts/pmc_summary.py gpurun_out/prof ${T}_cfg1 > gpurun_out/prof/${T}_cfg1_pmc_summary.txt && echo pmc ok
