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


def _lanewise_dw(G, X):
    """The MX dW as the kernel forms it (cvae_wgrad.h mx_dw_chunk): per 128-row chunk of the batch,
    lane r + 16j holds as byte quarter h the 8 rows 32·(2(h >> 1) + (j >> 1)) + 8·(2(h & 1) + (j & 1))
    + e of feature r (G: an output, X: an input); the instruction's block b of feature r is quarters
    2(b >> 1), +1 of the lanes j = 2(b & 1), +1; k = 134 − biased exponent of the block max."""
    B = G.shape[0]
    Bk = (B + 127) // 128 * 128

    def conv(A):
        F = A.shape[1]
        Ap = np.zeros((Bk, F), np.float32)
        Ap[:B] = A
        out = np.zeros((Bk, F))
        for c in range(Bk // 128):
            for b in range(4):
                rows = [128 * c + 32 * (2 * (h >> 1) + (j >> 1)) + 8 * (2 * (h & 1) + (j & 1)) + e
                        for h in (2 * (b >> 1), 2 * (b >> 1) + 1) for j in (2 * (b & 1), 2 * (b & 1) + 1)
                        for e in range(8)]
                for f in range(F):
                    v = Ap[rows, f]
                    m = float(np.abs(v).max())
                    eb = int((np.float32(m).view(np.uint32) >> 23) & 0xFF)
                    k = min(134 - eb, 126) if eb > 0 else 0
                    out[rows, f] = cvae_np.e4m3(v * np.float32(2.0 ** k)).astype(np.float64) * 2.0 ** -k
        return out
    return conv(G).T @ conv(X)


@pytest.mark.parametrize("B,N,K", [(128, 32, 64), (256, 16, 40), (200, 8, 24)])
def test_mx_dw_blocks_are_the_lanes(B, N, K):
    """oracle.cvae_np.mx_dw's reshape blocks (32 consecutive batch rows per feature) are exactly
    the blocks the lane assignment of the MX dW kernel forms; a ragged batch pads whole blocks
    with zero rows; e4m3 rounding of both operands (each element within half an e4m3 ulp, 3 %) stays
    within 8 % rel-L2 of the exact product."""
    rng = np.random.default_rng(B + N)
    G = cvae_np.bf16(rng.standard_normal((B, N)).astype(np.float32) * 1e-5)
    G[:, 0] *= 3e3            # a feature spanning 10^3 within a block (dL/drecon's start term)
    G[40:72] = 0.0            # an all-zero block
    X = cvae_np.bf16(np.maximum(rng.standard_normal((B, K)), 0).astype(np.float32))
    got = cvae_np.mx_dw(G, X)
    want = _lanewise_dw(G, X)
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-12)
    exact = G.astype(np.float64).T @ X
    err = np.linalg.norm(got - exact) / np.linalg.norm(exact)
    assert err < 0.08, err


def test_mxw_layers_cfg5():
    """Every cfg5 layer but the K=2 condition layer has a padded K that is a multiple of 64: its dW
    runs on the MX path's 32 × 64 tiles."""
    rng = np.random.default_rng(0)
    shapes = {"condition_encoder.0": (128, 2), "condition_encoder.2": (128, 128), "encoder.1": (128, 1200),
              "fc_mu": (512, 256), "fc_logvar": (512, 256), "decoder.0": (128, 640), "decoder.14": (1200, 128)}
    shapes.update({f"encoder.{2 * i + 1}": (128, 128) for i in range(1, 8)})
    shapes.update({f"decoder.{2 * i}": (128, 128) for i in range(1, 7)})
    p = {k + ".weight": rng.standard_normal(s).astype(np.float32) for k, s in shapes.items()}
    got = cvae_np.mxw_layers(p, 8, 8)
    assert "condition_encoder.0" not in got and len(got) == len(shapes) - 1
