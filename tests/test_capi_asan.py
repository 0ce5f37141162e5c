"""The C-ABI's host code under AddressSanitizer (auxiliary subsystems: "-fsanitize=address
host build of the C-ABI shim"; CPU only).

cvae_amd._build.build_asan compiles csrc/cvae_capi.hip with ``-Xarch_host -fsanitize=address`` into
build/asan/ (GPU AddressSanitizer is not available on this pool, so the device code stays
uninstrumented) and links tests/asan/capi_host_check.c against it.  The checker drives the host
logic every entry point has without a GPU — the planner over the BASELINE shapes and invalid ones,
NULL / bad-argument validation, error strings, cvae_create's failure path — and exits non-zero on a
failed expectation; ASan aborts it on any heap / stack error or leak.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_capi_host_code_is_asan_clean():
    from cvae_amd._build import build_asan
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc")
    so, exe = build_asan(os.path.join(ROOT, "build", "asan"))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "capi host check ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "ERROR: LeakSanitizer" not in r.stderr
