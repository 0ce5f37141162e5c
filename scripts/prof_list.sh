mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1 || true
grep -iE "ICACHE|IFETCH|WAIT|SQ_INSTS|SQ_BUSY|SQ_WAVE|LDS_BANK|SQ_INST_LEVEL|VMEM|TA_BUSY|SQ_ACTIVE" $GRAFT_REPO_ROOT/gpurun_out/counters.txt | head -120
