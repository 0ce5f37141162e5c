#!/bin/bash
# Round evidence on one MI355X (TAG=r04b ...): the whole -m gpu suite, smoke(), the driver's exact
# bench command (twice) beside a 200-step line, the other workloads' lines, the N>1 path rehearsed on
# the one GPU (2 and 4 ranks), a rocprofv3 kernel trace of the driver's command and the PMC passes
# (SQ instruction mix, HBM traffic, L2 hit/miss).  Every GPU step has its own limit; the script
# stops at the first failure.  SKIP_TESTS=1 skips the suite; PASSES overrides the PMC pass list.
set -u
T=${TAG:-r06z}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
fi
for r in a b; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_$r.json 2> $OUT/bench_s20_$r.err || exit 1
done
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline"
$B --steps 200 --warmup 20 > $OUT/bench_s200.json 2> $OUT/bench_s200.err &&
$B --steps 200 --warmup 20 --dp > $OUT/bench_dp.json 2> $OUT/bench_dp.err &&
$B --steps 200 --warmup 20 --dp --buckets 2 > $OUT/bench_dp_b2.json 2> $OUT/bench_dp_b2.err &&
$B --steps 200 --warmup 20 --workload cfg4 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err &&
$B --steps 100 --warmup 10 --workload wide > $OUT/bench_wide_bf16.json 2> $OUT/bench_wide_bf16.err &&
$B --steps 100 --warmup 10 --workload wide --dtype fp8 > $OUT/bench_wide_fp8.json 2> $OUT/bench_wide_fp8.err &&
CVAE_FP8_DW=mx $B --steps 100 --warmup 10 --workload wide --dtype fp8 > $OUT/bench_wide_fp8_mxdw.json 2> $OUT/bench_wide_fp8_mxdw.err &&
timeout -k 10 180 python3 bench.py --workload cfg1 --steps 50 --warmup 5 > $OUT/bench_cfg1.json 2> $OUT/bench_cfg1.err || { tail -5 $OUT/*.err; exit 1; }
# the N > 1 path rehearsed on the one GPU: bench.py starting its own N ranks (the plain --gpus N form),
# and once under torch.distributed.run (the driver's form)
for n in 2 4 8; do
  CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 timeout -k 10 400 python3 bench.py --gpus $n --steps 20 --warmup 5 \
    > $OUT/bench_share$n.json 2> $OUT/bench_share$n.err || { tail -5 $OUT/bench_share$n.err; exit 1; }
done
CVAE_BENCH_SHARE_GPU=1 CVAE_PX_TIMEOUT_MS=30000 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29582 bench.py --gpus 2 --steps 20 --warmup 5 \
  > $OUT/bench_share2_torchrun.json 2> $OUT/bench_share2_torchrun.err || { tail -5 $OUT/bench_share2_torchrun.err; exit 1; }
for f in $OUT/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'),r['frac'])"; done
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
# kernel trace of the driver's exact command (program directly after --)
P=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o ${T}_driver_trace -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $P/${T}_driver_trace.log 2>&1 || exit 1
echo driver trace ok
cd $GRAFT_REPO_ROOT
TAG=${T}_cfg2 PASSES=${PASSES:-sq1,sq2,ta,tcc,fetch,write} STEPS=100 bash scripts/profile.sh || exit 1
python3 scripts/pmc_traffic.py gpurun_out/prof ${T}_cfg2 gpurun_out/prof/${T}_traffic.json 1024 bf16 > /dev/null &&
python3 scripts/pmc_summary.py gpurun_out/prof ${T}_cfg2 > gpurun_out/prof/${T}_cfg2_pmc_summary.txt && echo pmc ok &&
# BASELINE cfg5 in e4m3: instruction mix, L2 hit/miss and HBM traffic of the wide chain and its dW
TAG=${T}_wfp8 PASSES=sq2,tcc,fetch,write STEPS=50 BENCH_EXTRA="--workload wide --dtype fp8" bash scripts/profile.sh &&
python3 scripts/pmc_traffic.py gpurun_out/prof ${T}_wfp8 gpurun_out/prof/${T}_wfp8_traffic.json 1024 fp8 > /dev/null &&
python3 scripts/pmc_summary.py gpurun_out/prof ${T}_wfp8 > gpurun_out/prof/${T}_wfp8_pmc_summary.txt && echo pmc wfp8 ok
