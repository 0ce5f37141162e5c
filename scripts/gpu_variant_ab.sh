#!/bin/bash
# GPU box: bench A/B of the current library against diagnostic builds (names in $VARIANTS, files
# $DIR/<name>.so, default build/diag) and environment settings ($ENVS: space-separated VAR=value
# items, each one variant), alternating $REPS times.  Workload: cfg2 (default), the wide shape
# ($WIDE=1, $DT=bf16|fp8) or any bench arguments in $EXTRA (e.g. "--workload cfg1").
set -u
O=${O:-gpurun_out/vab}; mkdir -p $O
DIR=${DIR:-build/diag}
EX="${EXTRA:-}"; [ "${WIDE:-0}" = 1 ] && EX="--workload wide --dtype ${DT:-bf16} --steps 100 --warmup 10"
B="timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 400 $EX"
for i in $(seq 1 ${REPS:-2}); do
  $B > $O/base$i.json 2> $O/base$i.err || exit 1
  for v in ${VARIANTS:-}; do CVAE_LIB=$PWD/$DIR/$v.so $B > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -3 $O/${v}_$i.err; exit 1; }; done
  for e in ${ENVS:-}; do env $e $B > $O/${e//=/_}_$i.json 2> $O/${e//=/_}_$i.err || { tail -3 $O/${e//=/_}_$i.err; exit 1; }; done
done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['kernels_ms'])"; done
