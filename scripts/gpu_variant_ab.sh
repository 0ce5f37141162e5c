#!/bin/bash
# GPU box: bench A/B of the current library against diagnostic builds (names in $VARIANTS),
# alternating, cfg2 (default) and optionally the wide shape ($WIDE=1).
set -u
O=${O:-gpurun_out/vab}; mkdir -p $O
EX=""; [ "${WIDE:-0}" = 1 ] && EX="--workload wide --dtype ${DT:-bf16} --steps 100 --warmup 10"
B="timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 400 $EX"
for i in 1 2; do
  $B > $O/base$i.json 2> $O/base$i.err || exit 1
  for v in $VARIANTS; do CVAE_LIB=$PWD/build/diag/$v.so $B > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -3 $O/${v}_$i.err; exit 1; }; done
done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernels_ms'])"; done
