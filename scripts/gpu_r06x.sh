set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06x; mkdir -p $O
CVAE_F32_SPREAD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_f32chain.py -k rows4 > $O/pytest_spread1.log 2>&1 || { tail -30 $O/pytest_spread1.log; exit 1; }
tail -1 $O/pytest_spread1.log
for i in 1 2; do
  for sp in 8 1 2; do
    CVAE_F32_SPREAD=$sp timeout -k 10 120 python3 bench.py --no-cpu-baseline --workload cfg1 --steps 400 --warmup 20 > $O/cfg1_s${sp}_$i.json 2> $O/cfg1_s${sp}_$i.err || exit 1
  done
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
