#!/bin/bash
# The -m gpu suite and smoke() on one MI355X (TAG=...): one pytest process, each test under a time limit.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-suite}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v -x -rP --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
