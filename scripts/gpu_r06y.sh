#!/bin/bash
# round 6: the 4-row chain's k-group sums by row swaps (default) vs the ds_bpermute butterfly
# (build/dx/kredshfl.so): probe, parity, cfg1 A/B at 400 steps
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06y2; mkdir -p $O
timeout -k 10 60 ./scripts/ubench/mfma4x4_layout > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_f32chain.py tests/test_hip_parity.py -k "f32 or traj20 or ragged or fixed_weights or epoch_chunks" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in base kredshfl; do
    L=""; [ $v != base ] && L="CVAE_LIB=$PWD/build/dx/$v.so"
    env $L timeout -k 10 120 python3 bench.py --no-cpu-baseline --workload cfg1 --steps 400 --warmup 20 > $O/cfg1_${v}_$i.json 2> $O/cfg1_${v}_$i.err || exit 1
  done
done
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline'].get('kernels_ms'))"; done
