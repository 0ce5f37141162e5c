set -u
O=gpurun_out/g5; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -q -k "fp8 or wide" --timeout 280 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
WIDE=1 SUB=1 DT=fp8 CVAE_LIB=$PWD/build/diag/wsub.so timeout -k 10 120 python3 scripts/diag_stamps.py > $O/substamps_wide_fp8.txt 2>&1 || { tail $O/substamps_wide_fp8.txt; exit 1; }
sed -n 20,40p $O/substamps_wide_fp8.txt | cut -c1-60
B="timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 --workload wide"
for i in 1 2; do $B --dtype fp8 > $O/wide_fp8_$i.json 2> $O/wide_fp8_$i.err || { tail -5 $O/wide_fp8_$i.err; exit 1; }; done
for f in $O/wide_*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
