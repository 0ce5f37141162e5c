set -u
O=gpurun_out/g1; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dp_autograd.py tests/test_train_dp.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/dp_tests.log 2>&1 || { tail -30 $O/dp_tests.log; exit 1; }
tail -2 $O/dp_tests.log
B="timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 --dp"
for i in 1 2; do
  $B > $O/dp_$i.json 2> $O/dp_$i.err && $B --buckets 2 > $O/dp_b2_$i.json 2> $O/dp_b2_$i.err && CVAE_GENERIC_BUCKETS=1 $B --buckets 2 > $O/dp_b2gen_$i.json 2> $O/dp_b2gen_$i.err || { tail -5 $O/*.err; exit 1; }
done
for f in $O/dp*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
