#!/bin/bash
# GPU box: rocprofv3 kernel traces of the final cfg5 wide chain (bf16, fp8) and the cfg2 default.
set -u
export TMPDIR=/tmp
TAG=r02l_wide_bf16 BENCH_EXTRA="--workload wide" PASSES=trace,fetch,write STEPS=50 bash scripts/profile.sh || exit 1
TAG=r02l_wide_fp8 BENCH_EXTRA="--workload wide --dtype fp8" PASSES=trace,sq2 STEPS=50 bash scripts/profile.sh || exit 1
TAG=r02l_cfg2 PASSES=trace STEPS=100 bash scripts/profile.sh || exit 1
cd $GRAFT_REPO_ROOT && python scripts/pmc_summary.py gpurun_out/prof r02l_wide_fp8 > gpurun_out/prof/r02l_wide_fp8_pmc_summary.txt
