#!/bin/bash
# GPU box: round-1 final profiles — cfg2 trace (default bench) and cfg5 bf16 vs fp8 trace + instruction mix.
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r01i STEPS=100 PASSES=trace bash scripts/profile.sh || exit $?
TAG=r01i_wide_bf16 STEPS=50 PASSES=trace,sq2 BENCH_EXTRA="--workload wide --dtype bf16" bash scripts/profile.sh || exit $?
TAG=r01i_wide_fp8 STEPS=50 PASSES=trace,sq2 BENCH_EXTRA="--workload wide --dtype fp8" bash scripts/profile.sh || exit $?
