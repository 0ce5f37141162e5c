#!/bin/bash
# GPU box: rocprofv3 kernel trace (+stats) and PMC passes of the bench step (1 GPU).
# Writes gpurun_out/prof/<tag>_*; each pass has its own time limit; stop at first failure.
set -u
TAG=${TAG:-r01}
STEPS=${STEPS:-50}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps $STEPS --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o ${TAG}_trace -- python3 $BENCH > $OUT/${TAG}_trace.log 2>&1 || exit $?
echo trace ok
i=0
for grp in "${PMC_GROUPS[@]:-}"; do :; done
run_pmc() {
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $1 --output-format csv -d $OUT -o ${TAG}_pmc$i -- python3 $BENCH > $OUT/${TAG}_pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; return $rc
}
run_pmc "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS SQ_IFETCH" || exit $?
run_pmc "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INSTS_BRANCH" || exit $?
run_pmc "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_IFETCH_LEVEL" || exit $?
run_pmc "FETCH_SIZE" || exit $?
run_pmc "WRITE_SIZE" || exit $?
ls $OUT
