#!/bin/bash
# GPU box: rocprofv3 trace + PMC passes of the final default cfg2 step (ring chain) and cfg5 fp8.
set -u
export TMPDIR=/tmp
TAG=r02m_cfg2 PASSES=trace,sq1,sq2,fetch,write STEPS=100 bash scripts/profile.sh || exit 1
TAG=r02m_wide_fp8 BENCH_EXTRA="--workload wide --dtype fp8" PASSES=trace STEPS=50 bash scripts/profile.sh || exit 1
cd $GRAFT_REPO_ROOT && python scripts/pmc_summary.py gpurun_out/prof r02m_cfg2 > gpurun_out/prof/r02m_cfg2_pmc_summary.txt
