"""Build the HIP C-ABI library (gfx950 only) in-tree.

``python -m cvae_amd._build`` or ``__graft_entry__.build()``.  The .so lands next
to this file so it travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
LIB = os.environ.get("CVAE_LIB") or os.path.join(HERE, "libcvae_hip.so")  # CVAE_LIB: diagnostic builds only
SOURCES = ["cvae_capi.hip"]
HEADERS = ["cvae_device.h", "cvae_rowchain.h", "cvae_fastchain.h", "cvae_fastwgrad.h", "cvae_wgrad.h", "cvae_loss.h",
           "cvae_extract.h", "cvae_mpc.h", "cvae_widechain.h", "cvae_peer.h", "cvae_widewgrad.h",
           "cvae_f32chain.h", "cvae_f32wgrad.h"]
ARCH = "gfx950"


def _inputs():
    root = os.path.dirname(os.path.dirname(HERE))
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    files.append(os.path.join(root, "include", "cvae.h"))
    return files


def _command(out):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-Wno-pass-failed", "-mllvm", "-amdgpu-mfma-vgpr-form",
           "-mllvm", "-amdgpu-kernarg-preload-count=16", "-o", out]
    cmd += os.environ.get("CVAE_EXTRA_FLAGS", "").split()  # diagnostic builds only (with CVAE_LIB)
    return cmd + [os.path.join(CSRC, s) for s in SOURCES] + ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def source_digest() -> str:
    """sha256 over every input's bytes and the compile flags: what the library was built from.
    Kept beside the library (``<lib>.sha256``) so a library is rebuilt when its sources differ,
    whatever the files' timestamps say."""
    h = hashlib.sha256()
    for f in _inputs():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(_command("")[1:]).encode())
    return h.hexdigest()


def _stamp():
    return LIB + ".sha256"


def needs_build() -> bool:
    if not os.path.exists(LIB) or not os.path.exists(_stamp()):
        return True
    with open(_stamp()) as f:
        return f.read().strip() != source_digest()


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile when the library is missing or was built from other sources (content digest);
    with ``verbose`` say which (the hipcc command, or "up to date")."""
    digest = source_digest()
    if not force and not needs_build():
        if verbose:
            print(f"cvae_amd: {LIB} up to date (sources sha256 {digest[:16]})", file=sys.stderr)
        return LIB
    tmp = LIB + ".tmp"
    cmd = _command(tmp)
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, LIB)
    with open(_stamp(), "w") as f:
        f.write(digest + "\n")
    if verbose:
        print(f"cvae_amd: built {LIB} (sources sha256 {digest[:16]})", file=sys.stderr)
    return LIB


def build_asan(out_dir, verbose=False) -> tuple:
    """The C-ABI with its HOST code under AddressSanitizer (tests/test_capi_asan.py):
    ``-Xarch_host -fsanitize=address`` (GPU AddressSanitizer is not available here; the device code
    is built as usual, uninstrumented), plus the host-side checker tests/asan/capi_host_check.c
    linked against it.  Rebuilt when a source is newer.  Returns (library, checker) paths."""
    root = os.path.dirname(os.path.dirname(HERE))
    os.makedirs(out_dir, exist_ok=True)
    so = os.path.join(out_dir, "libcvae_asan.so")
    exe = os.path.join(out_dir, "capi_host_check")
    drv = os.path.join(root, "tests", "asan", "capi_host_check.c")
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not os.path.exists(so) or any(os.path.getmtime(f) > os.path.getmtime(so) for f in _inputs()):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result",
               "-Wno-pass-failed", "-mllvm", "-amdgpu-mfma-vgpr-form", "-Xarch_host", "-fsanitize=address",
               "-Xarch_host", "-fno-omit-frame-pointer", "-o", so + ".tmp", os.path.join(CSRC, "cvae_capi.hip"),
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, cwd=CSRC)
        os.replace(so + ".tmp", so)
    if not os.path.exists(exe) or max(os.path.getmtime(so), os.path.getmtime(drv)) > os.path.getmtime(exe):
        clang = os.path.join(os.path.dirname(os.path.realpath(hipcc)), "..", "llvm", "bin", "clang")
        if not os.path.exists(clang):
            clang = "/opt/rocm/llvm/bin/clang"
        subprocess.run([clang, "-g", "-O1", "-fsanitize=address", "-fno-omit-frame-pointer", "-o", exe, drv,
                        "-L" + out_dir, "-lcvae_asan", "-Wl,-rpath," + out_dir], check=True)
    return so, exe


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
