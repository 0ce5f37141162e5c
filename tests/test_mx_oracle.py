"""The oracle's restatement of the wide chain's e4m3 dX GEMM with MX row-block scales
(oracle/cvae_np.py mx_dx ↔ csrc/cvae_widechain.h gemm_mxb / mx_block), checked on CPU against a
lane-by-lane restatement of the kernel: lane r + 16q of K-pair group g holds, as byte quarter h, the
8 values of chunk 4g + h at chunk positions frag_k(q, e) (cvae_device.h: 4q + e, 16 + 4q + e); the
instruction's MX block b of row r is quarters 2(b >> 1), 2(b >> 1) + 1 of the lanes q = 2(b & 1),
2(b & 1) + 1 (the mapping scripts/ubench/mxscale.hip measured on the GPU), so k = 134 − biased
exponent of the block max, 2^k·g is converted to e4m3 and multiplied with unit-scaled e4m3(s·W)
under the E8M0 scales 2^−k and 1/s.  The blocks a reshape forms in mx_dx must be exactly these."""
import numpy as np
import pytest

from oracle import cvae_np


def _frag_k(q, e):
    return 4 * q + e if e < 4 else 12 + 4 * q + e


def _lanewise(G, W, s):
    B, N = G.shape
    K = W.shape[1]
    groups = (N + 127) // 128
    w8 = cvae_np.e4m3(W.astype(np.float32) * s).astype(np.float64) / s
    out = np.zeros((B, K))
    for r in range(B):
        for g in range(groups):
            for b in range(4):
                pos = [128 * g + 32 * h + _frag_k(q, e) for h in (2 * (b >> 1), 2 * (b >> 1) + 1)
                       for q in (2 * (b & 1), 2 * (b & 1) + 1) for e in range(8)]
                pos = [p for p in pos if p < N]
                if not pos:
                    continue
                v = G[r, pos].astype(np.float32)
                m = float(np.abs(v).max())
                eb = int((np.float32(m).view(np.uint32) >> 23) & 0xFF)
                k = min(134 - eb, 126) if eb > 0 else 0
                x8 = cvae_np.e4m3(v * np.float32(2.0 ** k)).astype(np.float64) * 2.0 ** -k
                out[r] += x8 @ w8[pos]
    return out


@pytest.mark.parametrize("N,K", [(128, 640), (1200, 128), (512, 256)])
def test_mx_dx_blocks_are_the_lanes(N, K):
    rng = np.random.default_rng(N)
    G = cvae_np.bf16(rng.standard_normal((16, N)).astype(np.float32) * 1e-6)
    G[:, 1:3] *= 3e3           # the start-term outliers of dL/drecon (a 10^3-10^4 range in a row)
    G[5] = 0.0                 # a padding row: all-zero blocks
    W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
    s = cvae_np.f8_scale(W)
    got = cvae_np.mx_dx(G, W, s)
    want = _lanewise(G, W, s)
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-12)
    assert not got[5].any()
    exact = G.astype(np.float64) @ W
    err = np.linalg.norm(got - exact) / np.linalg.norm(exact)
    assert err < 0.06, err     # e4m3 rounding of both operands (3 mantissa bits)


def test_fp8b_layers_cfg5():
    """The f8b set at BASELINE cfg5 is the last decoder layer, decoder L0 and fc (build_plan's rule)."""
    rng = np.random.default_rng(0)
    H, Z, I, ne, nd = 128, 512, 1200, 8, 8
    p = {"fc_mu.weight": rng.standard_normal((Z, 2 * H)), "fc_logvar.weight": rng.standard_normal((Z, 2 * H)),
         "condition_encoder.0.weight": rng.standard_normal((H, 2)),
         "condition_encoder.2.weight": rng.standard_normal((H, H))}
    for i in range(ne):
        p[f"encoder.{2 * i + 1}.weight"] = rng.standard_normal((H, I if i == 0 else H))
    for i in range(nd):
        p[f"decoder.{2 * i}.weight"] = rng.standard_normal((I if i == nd - 1 else H, Z + H if i == 0 else H))
    f8b = cvae_np.fp8b_layers(p, 200, 6, Z, H, ne, nd)
    assert sorted(f8b) == ["decoder.0", "decoder.14", "fc_logvar", "fc_mu"]
    assert f8b["fc_mu"] == f8b["fc_logvar"]
    assert not cvae_np.fp8b_layers(p | {"decoder.6.weight": rng.standard_normal((600, 128))}, 100, 6, 8, H, 4, 4)
