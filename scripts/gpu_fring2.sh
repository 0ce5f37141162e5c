#!/bin/bash
# Round 4 (commit dc3e266, the kernel removed since): the one-launch ring step with the decoder tiles gated on the decoder rows (CVAE_FUSE_RING=2, 3)
# against the two-launch step (0) and the round-3 one-launch form (1): parity tests, then the
# bench alternating the four (200 steps, twice), and the per-step stamps of mode 2.
set -u
O=gpurun_out/fring2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_hip_parity.py -m gpu -x -q -k fused_ring --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 200 --warmup 20"
for i in 1 2; do
  for m in 0 1 2 3; do CVAE_FUSE_RING=$m $B > $O/m${m}_$i.json 2> $O/m${m}_$i.err || { tail -5 $O/m${m}_$i.err; exit 1; }; done
done
for f in $O/m*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('kernels_ms'))"; done
RING=1 CVAE_FUSE_RING=2 CVAE_LIB=$PWD/build/diag/fr2st.so timeout -k 10 120 python3 scripts/diag_stamps.py > $O/stamps_m2.txt 2>&1 || { tail $O/stamps_m2.txt; exit 1; }
tail -12 $O/stamps_m2.txt
