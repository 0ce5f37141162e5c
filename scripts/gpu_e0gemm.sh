#!/bin/bash
# The encoder-L1 GEMM in isolation (scripts/ubench/e0gemm.hip, built here on the CPU): time and
# rooflines at M = 2^16..2^20 rows, then one PMC pass (MFMA busy) and one traffic pass at 2^18.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/e0gemm
mkdir -p $OUT
B=$GRAFT_REPO_ROOT/scripts/ubench/e0gemm
for M in 65536 262144 1048576; do
  timeout -k 10 60 $B $M 50 > $OUT/run_$M.json 2> $OUT/run_$M.err || { cat $OUT/run_$M.err; exit 1; }
  cat $OUT/run_$M.json
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT -o pmc_mfma -- $B 262144 5 > $OUT/pmc_mfma.log 2>&1 || { tail -5 $OUT/pmc_mfma.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o pmc_fetch -- $B 262144 5 > $OUT/pmc_fetch.log 2>&1 || { tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o pmc_write -- $B 262144 5 > $OUT/pmc_write.log 2>&1 || { tail -5 $OUT/pmc_write.log; exit 1; }
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- $B 262144 20 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
find $OUT -name "*.csv" | head
