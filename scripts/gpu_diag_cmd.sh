mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
CVAE_LIB=build/diag/stamps.so timeout -k 10 120 python scripts/diag_stamps.py > gpurun_out/stamps.log 2>&1; rc=$?; echo "stamps rc=$rc"; cat gpurun_out/stamps.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernels_ms'])"
