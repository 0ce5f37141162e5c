#!/bin/bash
# GPU box: wide-chain tests (bf16 + the fp8 form) → cfg5 benches bf16 / fp8.
set -u
O=gpurun_out/wf8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "${K:-wide or fp8}" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert|rel-L2" $O/pytest.log | head -30; exit $rc; }
grep -E "rel-L2|deviation" $O/pytest.log | head
B="timeout -k 10 180 python -u bench.py --no-cpu-baseline --workload wide --steps 100 --warmup 10"
$B > $O/bench_wide_bf16.json 2> $O/bench_wide_bf16.err && $B --dtype fp8 > $O/bench_wide_fp8.json 2> $O/bench_wide_fp8.err || { tail -5 $O/*.err; exit 1; }
for f in $O/bench_*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernels_ms'],r.get('kernels_back_to_back_ms'))"; done
