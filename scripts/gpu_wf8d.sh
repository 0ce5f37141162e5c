#!/bin/bash
set -u
mkdir -p gpurun_out/wst && bash scripts/gpu_wstamps.sh > gpurun_out/wst/paste.txt && grep -h -A3 "^wgrad" gpurun_out/wst/wide_bf16.txt gpurun_out/wst/wide_fp8.txt | cut -c1-250
