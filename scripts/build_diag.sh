#!/bin/bash
# Build diagnostic variants of the library here (CPU): build/diag/<name>.so, one per "name:FLAGS" arg.
# e.g. bash scripts/build_diag.sh stamps:-DCVAE_DIAG_STAMPS=1 sub:-DCVAE_DIAG_SUB=1
cd "$(dirname "$0")/.."
mkdir -p build/diag
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( CVAE_LIB=$PWD/build/diag/$name.so CVAE_EXTRA_FLAGS="$flags" python -c "
import sys; sys.path.insert(0, 'defensive-model-vae_amd')
from cvae_amd import _build; _build.build(force=True)" && echo "built $name" ) &
done
wait
