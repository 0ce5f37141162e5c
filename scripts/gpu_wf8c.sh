#!/bin/bash
set -u
K="wide or fp8" bash scripts/gpu_wide_fp8.sh && bash scripts/gpu_wsub.sh
