"""Register and scratch budgets of the built library's hot kernels (CPU only: reads the gfx950 code
object's metadata notes, launches nothing).

* The reference architecture's ring chain (cfg2 and cfg4 instantiations of
  wchain::widechain_kernel) must stay within 128 VGPRs: a chain block then shares a CU with a dW-tile
  block of another process.  Ranks time-sharing one GPU (tests/test_gpu_peer.py) depend on it — a
  138-VGPR build starved the other rank's peer-exchange kernel into its time-out (round 3).
* The peer-exchange and one-launch kernels promise every block resident at two workgroups per CU
  (<= 128 VGPRs).
* No hot kernel spills to scratch.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import kernel_resources  # noqa: E402

LIB = kernel_resources.LIB
RING = "Arch<100, 6, 8, 4, 4"


@pytest.fixture(scope="module")
def res():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    r = kernel_resources.resources(LIB)
    if not r:
        pytest.skip("no gfx950 code object metadata readable")
    return r


def _pick(res, *subs):
    return [k for k in res if all(s in k["demangled"] for s in subs)]


def test_ring_chain_fits_128_vgprs_without_scratch(res):
    ks = _pick(res, "widechain_kernel", RING)
    # widechain_kernel<Arch<...>, TAP, XB>: XB = bf16 rows only (the fp32-row loads compiled out)
    tap = [k for k in ks if ">, true, false>(" in k["demangled"]]
    prod = [k for k in ks if k not in tap]
    # cfg2 and cfg4 (class embedding), each with both row formats and bf16 rows only
    assert len(prod) == 4 and sum(", false, true>(" in k["demangled"] for k in prod) == 2, [k["demangled"] for k in ks]
    assert len(tap) == 1, [k["demangled"] for k in ks]   # cfg2's parity-tap form (cvae_tap_outputs)
    for k in prod:
        assert k["vgpr"] <= 128 and k["scratch"] == 0, k
    assert tap[0]["scratch"] == 0, tap[0]


def test_two_blocks_per_cu_kernels_fit(res):
    for name in ("px_wgrad_kernel",):
        ks = _pick(res, name)
        assert ks, name
        for k in ks:
            # px_wgrad_kernel<19, true>: the tile loop of ranks SHARING one GPU (a rehearsal; one rank
            # per GPU runs <19, false>) may spill a few registers; it must still fit two per CU
            shared = ", true>(" in k["demangled"]
            assert k["vgpr"] <= 128 and (k["scratch"] == 0 or (shared and k["scratch"] <= 256)), k


def test_hot_kernels_do_not_spill(res):
    for name in ("widechain_kernel", "fastchain_kernel", "fastwgrad_kernel", "wgrad_kernel"):
        for k in _pick(res, name):
            if name == "wgrad_kernel" and "px_wgrad_kernel" in k["demangled"]:
                continue  # the exchange kernels: test_two_blocks_per_cu_kernels_fit
            assert k["scratch"] == 0, k
