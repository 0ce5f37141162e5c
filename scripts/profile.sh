#!/bin/bash
# GPU box: rocprofv3 kernel trace (+stats) and PMC passes of the bench step (1 GPU).
# Writes gpurun_out/prof/<TAG>_*; each pass has its own time limit; stops at the first failure.
# PASSES=trace,sq1,sq2,sq3,ta,tcc,fetch,write (default all)
set -u
TAG=${TAG:-r01}
STEPS=${STEPS:-50}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-b2b --steps $STEPS --warmup 5 ${BENCH_EXTRA:-}"  # BENCH_EXTRA: e.g. --workload wide --dtype fp8
P=${PASSES:-trace,sq1,sq2,sq3,ta,tcc,fetch,write}
has() { case ",$P," in *",$1,"*) return 0;; *) return 1;; esac; }
if has trace; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o ${TAG}_trace -- python3 $BENCH > $OUT/${TAG}_trace.log 2>&1 || exit $?
  echo trace ok
fi
run_pmc() {
  timeout -k 10 300 rocprofv3 --pmc $2 --output-format csv -d $OUT -o ${TAG}_pmc_$1 -- python3 $BENCH > $OUT/${TAG}_pmc_$1.log 2>&1
  rc=$?; echo "pmc $1 rc=$rc"; return $rc
}
has sq1 && { run_pmc sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS SQ_IFETCH" || exit $?; }
has sq2 && { run_pmc sq2 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" || exit $?; }
has sq3 && { run_pmc sq3 "SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_IFETCH_LEVEL SQ_ACTIVE_INST_LDS" || exit $?; }
has ta && { run_pmc ta "TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCC_WRITE_REQ" || exit $?; }
has tcc && { run_pmc tcc "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCP_TCC_READ_REQ_sum" || exit $?; }
has fetch && { run_pmc fetch "FETCH_SIZE" || exit $?; }
has write && { run_pmc write "WRITE_SIZE" || exit $?; }
ls $OUT | head -50
