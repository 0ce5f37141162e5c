#!/bin/bash
# Round 6 measurement set on one MI355X (TAG=r06x): the phase ubench kernel E (weights from a resident
# LDS image), the -m gpu suite, the wide fp8 / cfg2 sub-stamps, and an alternating A/B of the
# library against diagnostic builds in build/dx ($VARIANTS) at cfg2 and cfg5 fp8.  Every GPU step has
# its own limit; the script stops at the first failure.
set -u
T=${TAG:-r06x}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "${PHASE:-1}" = 1 ]; then timeout -k 10 60 ./scripts/ubench/phase E > $O/phase_e.txt 2>&1 || exit 1; cat $O/phase_e.txt; fi
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
if [ "${STAMPS:-1}" = 1 ]; then
  CVAE_LIB=$PWD/build/dx/stamps2.so WIDE=1 DT=fp8 SUB=1 timeout -k 10 120 python3 scripts/diag_stamps.py > $O/substamps_wide_fp8.txt 2>&1 || exit 1
  CVAE_LIB=$PWD/build/dx/stamps2.so RING=1 SUB=1 timeout -k 10 120 python3 scripts/diag_stamps.py > $O/substamps_cfg2.txt 2>&1 || exit 1
fi
for i in 1 2; do
  for v in base ${VARIANTS:-}; do
    L=""; [ $v != base ] && L="CVAE_LIB=$PWD/build/dx/$v.so"
    env $L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 200 --warmup 20 > $O/cfg2_${v}_$i.json 2> $O/cfg2_${v}_$i.err || { tail -3 $O/cfg2_${v}_$i.err; exit 1; }
    env $L timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-b2b --steps 100 --warmup 10 --workload wide --dtype fp8 > $O/wfp8_${v}_$i.json 2> $O/wfp8_${v}_$i.err || { tail -3 $O/wfp8_${v}_$i.err; exit 1; }
  done
done
for f in $O/cfg2_*.json $O/wfp8_*.json; do python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernels_ms'])"; done
