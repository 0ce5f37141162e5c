#!/bin/bash
# Build diagnostic variants of the library (here) — run scripts/diag_run.sh on the GPU box.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/diag
SRC=defensive-model-vae_amd/csrc/cvae_capi.hip
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-pass-failed"
hipcc $F -o build/diag/base.so $SRC &
hipcc $F -DCVAE_DIAG_NOSTORE=1 -o build/diag/nostore.so $SRC &
hipcc $F -DCVAE_DIAG_NOBIAS=1 -o build/diag/nobias.so $SRC &
hipcc $F -DCVAE_DIAG_NOSTORE=1 -DCVAE_DIAG_NOBIAS=1 -o build/diag/nostore_nobias.so $SRC &
wait
ls -la build/diag
