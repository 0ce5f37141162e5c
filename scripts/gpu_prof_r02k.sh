#!/bin/bash
# GPU box: round-2 profiles — cfg2 (fastchain default, ring opt-in) and cfg5 wide (bf16, fp8):
# rocprofv3 kernel trace + stats, and PMC passes (SQ instruction mix, HBM traffic) for cfg2.
set -u
export TMPDIR=/tmp
TAG=r02k_cfg2 PASSES=trace,sq1,sq2,fetch,write STEPS=100 bash scripts/profile.sh || exit 1
CVAE_RING=1 TAG=r02k_ring PASSES=trace,sq1,sq2,fetch,write STEPS=100 bash scripts/profile.sh || exit 1
TAG=r02k_wide_bf16 BENCH_EXTRA="--workload wide" PASSES=trace,sq2 STEPS=50 bash scripts/profile.sh || exit 1
TAG=r02k_wide_fp8 BENCH_EXTRA="--workload wide --dtype fp8" PASSES=trace,sq2 STEPS=50 bash scripts/profile.sh || exit 1
cd $GRAFT_REPO_ROOT && for t in r02k_cfg2 r02k_ring r02k_wide_bf16 r02k_wide_fp8; do python scripts/pmc_summary.py gpurun_out/prof $t > gpurun_out/prof/${t}_pmc_summary.txt; done
ls gpurun_out/prof | head -80
