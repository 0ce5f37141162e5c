#!/bin/bash
# Round 3: the one-launch ring step (cvae_fusedring.h) — parity tests, then a bench A/B against the
# two-launch step (CVAE_FUSE_RING=0/1 at handle creation), 200 steps and the driver's 20-step command.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-fring}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "fused_ring or ring_chain or fused_step_equals" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
B="timeout -k 10 120 python3 bench.py --no-cpu-baseline"
for i in 1 2; do
  for v in 0 1; do
    CVAE_FUSE_RING=$v $B --steps 200 --warmup 20 > $OUT/s200_f${v}_$i.json 2> $OUT/s200_f${v}_$i.err || { tail -5 $OUT/s200_f${v}_$i.err; exit 1; }
    CVAE_FUSE_RING=$v $B --steps 20 --warmup 5 > $OUT/s20_f${v}_$i.json 2> $OUT/s20_f${v}_$i.err || { tail -5 $OUT/s20_f${v}_$i.err; exit 1; }
  done
done
for f in $OUT/s*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'),r.get('kernels_back_to_back_ms'))"; done
