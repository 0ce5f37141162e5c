"""Build the HIP C-ABI library (gfx950 only) in-tree.

``python -m cvae_amd._build`` or ``__graft_entry__.build()``.  The .so lands next
to this file so it travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
LIB = os.environ.get("CVAE_LIB") or os.path.join(HERE, "libcvae_hip.so")  # CVAE_LIB: diagnostic builds only
SOURCES = ["cvae_capi.hip"]
HEADERS = ["cvae_device.h", "cvae_rowchain.h", "cvae_fastchain.h", "cvae_fastwgrad.h", "cvae_wgrad.h", "cvae_loss.h",
           "cvae_extract.h", "cvae_mpc.h", "cvae_widechain.h", "cvae_peer.h", "cvae_fusedring.h"]
ARCH = "gfx950"


def _inputs():
    root = os.path.dirname(os.path.dirname(HERE))
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    files.append(os.path.join(root, "include", "cvae.h"))
    return files


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(f) > t for f in _inputs())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = LIB + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-Wno-pass-failed", "-mllvm", "-amdgpu-mfma-vgpr-form",
           "-mllvm", "-amdgpu-kernarg-preload-count=16", "-o", tmp]
    cmd += os.environ.get("CVAE_EXTRA_FLAGS", "").split()  # diagnostic builds only (with CVAE_LIB)
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
