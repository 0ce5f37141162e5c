#!/bin/bash
# GPU box: the data-parallel step's structure at one rank (scripts/dp_overhead.py) and its kernel trace.
set -u
mkdir -p gpurun_out/dp; export TMPDIR=/tmp
timeout -k 10 240 python scripts/dp_overhead.py > gpurun_out/dp/dp_overhead.log 2>&1 || { tail -5 gpurun_out/dp/dp_overhead.log; exit 1; }
cat gpurun_out/dp/dp_overhead.log | tail -8
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dp -o dp_trace -- python3 $GRAFT_REPO_ROOT/scripts/dp_overhead.py > $GRAFT_REPO_ROOT/gpurun_out/dp/dp_trace.log 2>&1 || exit $?
