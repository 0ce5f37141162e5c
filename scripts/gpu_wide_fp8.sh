#!/bin/bash
# Round 4: the cfg5 e4m3 backward (MX row-block scales) — its parity tests, the wide bench lines
# (bf16 beside fp8, twice) and per-step stamps of the fp8 chain (diagnostic build).  Each GPU step
# has its own limit; the script stops at the first failure.
set -u
O=${O:-gpurun_out/wide_fp8}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -v -rP -k "fp8 or wide" \
  --timeout 280 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED" $O/tests.log | tail -20
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 --workload wide"
for i in 1 2; do
  $B > $O/wide_bf16_$i.json 2> $O/wide_bf16_$i.err && $B --dtype fp8 > $O/wide_fp8_$i.json 2> $O/wide_fp8_$i.err \
    || { tail -5 $O/*.err; exit 1; }
done
for f in $O/wide_*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
WIDE=1 DT=fp8 CVAE_LIB=$PWD/build/diag/wstamps.so timeout -k 10 120 python3 scripts/diag_stamps.py > $O/stamps_wide_fp8.txt 2>&1 || { tail $O/stamps_wide_fp8.txt; exit 1; }
WIDE=1 DT=bf16 CVAE_LIB=$PWD/build/diag/wstamps.so timeout -k 10 120 python3 scripts/diag_stamps.py > $O/stamps_wide_bf16.txt 2>&1 || { tail $O/stamps_wide_bf16.txt; exit 1; }
cat $O/stamps_wide_fp8.txt
