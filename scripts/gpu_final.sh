#!/bin/bash
# GPU box: the round-end set — full -m gpu suite, smoke(), default bench (with CPU baseline), the
# DP and wide bench lines.  Each step bounded; stops at the first failure.
set -u
O=gpurun_out/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
B="timeout -k 10 240 python -u bench.py"
$B > $O/bench_default.json 2> $O/bench_default.err &&
$B --steps 200 --no-cpu-baseline --dp > $O/bench_dp_graph8.json 2> $O/bench_dp.err &&
$B --steps 100 --warmup 10 --no-cpu-baseline --workload wide > $O/bench_wide_bf16.json 2> $O/bench_wide.err &&
$B --steps 100 --warmup 10 --no-cpu-baseline --workload wide --dtype fp8 > $O/bench_wide_fp8.json 2> $O/bench_wide_fp8.err || { tail -5 $O/*.err; exit 1; }
for f in $O/bench_*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernels_ms'],r.get('weight_stream',{}).get('achieved_GBps_per_CU'),d.get('cpu_baseline',{}).get('value'))"; done
