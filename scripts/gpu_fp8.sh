set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -k "fp8" > gpurun_out/pytest_fp8.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|fp8 cfg|passed|failed" gpurun_out/pytest_fp8.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for dt in bf16 fp8; do
timeout -k 10 200 python bench.py --workload wide --dtype $dt --no-cpu-baseline > gpurun_out/bench_wide_$dt.json 2>gpurun_out/bench_wide_$dt.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_wide_$dt.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_wide_$dt.json'));r=d['roofline'];print('$dt',d['value'],d['ms_per_step'],r['kernels_ms'])"
done
