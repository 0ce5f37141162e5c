#!/bin/bash
set -u
bash scripts/gpu_fring_stamps.sh > /dev/null 2>&1 || { echo stamps failed; tail gpurun_out/frst/*.txt; exit 1; }
tail -12 gpurun_out/frst/fring1.txt
TAG=fring2 bash scripts/gpu_fring.sh
