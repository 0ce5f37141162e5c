"""Analytic (hand-derived) forward/backward/Adam of the CVAE step in numpy — TEST INFRASTRUCTURE.

The HIP kernels implement the backward pass analytically (no autograd), so this
module restates exactly those formulas on the CPU and is checked against the
autograd goldens of the reference (``tests/test_oracle_golden.py``).  It also
serves as a float64 yardstick when calibrating the bf16 tolerances.

Formulas (reference lines cited per function):
  loss      Training_VAE.py:240-267
  dL/dr     = w_r·2(r−x)/(B·S·D)
              + [s=0, d∈{1,2}] w_s·2(r−x)/(2B)
              + [s=0, d=0]     w_t·2r/B
              + [d=0] w_t/(B(S−1)) · ([r_s > r_{s+1}] − [r_{s−1} > r_s])   (ReLU'(0)=0)
  dL/dmu    = w_k·mu/(B·Z) + dz
  dL/dlv    = w_k·½(e^lv − 1)/(B·Z) + dz·eps·½·e^{lv/2}
  Linear    dX = G·W,  dW = Gᵀ·X,  db = Σ_b G;  h_c collects two consumers
  Adam      torch/optim/adam.py ``_single_tensor_adam`` op order (lerp, mul+addcmul,
            sqrt/bias-correction, addcdiv)
"""
from __future__ import annotations

import numpy as np

KEYS_ORDER = None  # filled by param_keys()


def param_keys(n_enc=4, n_dec=4):
    """state_dict order of Training_VAE.py:132-167 (24 keys at 4+4)."""
    ks = ["condition_encoder.0", "condition_encoder.2"]
    ks += [f"encoder.{2 * i + 1}" for i in range(n_enc)]
    ks += ["fc_mu", "fc_logvar"]
    ks += [f"decoder.{2 * i}" for i in range(n_dec)]
    out = []
    for k in ks:
        out += [k + ".weight", k + ".bias"]
    return out


def bf16(a):
    """Round-to-nearest-even to bfloat16, returned as float32 (the kernels' operand rounding)."""
    a = np.ascontiguousarray(a, np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def _ident(a):
    return a


E4M3_MAX = 448.0


def e4m3(a):
    """Round-to-nearest-even to OCP fp8 e4m3 (saturated at ±448), returned as float32 — the
    rounding of v_cvt_pk_fp8_f32 behind the CVAE_FP8 kernels (cvae_device.h f8x8)."""
    import torch  # the e4m3 cast (torch.float8_e4m3fn) is the only use of torch here

    a = np.clip(np.ascontiguousarray(a, np.float32), -E4M3_MAX, E4M3_MAX)
    return torch.from_numpy(a).to(torch.float8_e4m3fn).float().numpy()


def f8_scale(*ws):
    """Per-layer power-of-two weight scale of the fp8 operand: 2^floor(log2(448 / (4·max|W|)))
    (cvae_wgrad.h f8_scale_kernel; fc_mu and fc_logvar share one, they are one fused layer)."""
    amax = max(float(np.abs(w).max()) for w in ws)
    return np.float32(2.0 ** np.floor(np.log2(E4M3_MAX / (4.0 * amax)))) if amax > 0 else np.float32(1.0)


def _lin(x, p, name, q=_ident, sc=None):
    if sc is not None:  # fp8 forward GEMM: e4m3(bf16 activations) x e4m3(s·W), result / s
        w8 = e4m3(p[name + ".weight"].astype(np.float32) * sc)
        return (e4m3(q(x)) @ w8.T) / sc + p[name + ".bias"]
    return q(x) @ q(p[name + ".weight"]).T + p[name + ".bias"]


def fp8_layers(p, seq_len, dim, latent_dim, hidden_dim=128, n_enc=4, n_dec=4):
    """{layer name: scale} of the layers the CVAE_FP8 path runs in e4m3: padded K % 64 == 0
    (cvae_capi.hip build_plan), K = the layer's input width."""
    I, H, Z = seq_len * dim, hidden_dim, latent_dim
    ks = {"condition_encoder.0": 2, "condition_encoder.2": H, "fc": 2 * H}
    for i in range(n_enc):
        ks[f"encoder.{2 * i + 1}"] = I if i == 0 else H
    for i in range(n_dec):
        ks[f"decoder.{2 * i}"] = Z + H if i == 0 else H
    out = {}
    for name, k in ks.items():
        if (k + 31) // 32 * 32 % 64:
            continue
        if name == "fc":
            s = f8_scale(p["fc_mu.weight"], p["fc_logvar.weight"])
            out["fc_mu"] = out["fc_logvar"] = s
        else:
            out[name] = f8_scale(p[name + ".weight"])
    return out


def fp8b_layers(p, seq_len, dim, latent_dim, hidden_dim=128, n_enc=4, n_dec=4):
    """{layer name: scale} of the layers whose dX GEMM the CVAE_FP8 wide chain runs in e4m3 with MX
    row-block scales (cvae_capi.hip build_plan LayerDev::f8b, cvae_widechain.h Arch::f8b): an e4m3
    forward operand (padded K % 64 == 0), the backward K (the padded outputs) a multiple of 64, a dX
    at all (not condition_encoder.0 / encoder.1) and a padded extent of >= 512 on either side — at
    BASELINE cfg5 the last decoder layer, decoder.0 and fc.  Only the wide chain runs them (the
    generic interpreter's fp8 backward stays bf16)."""
    I, H, Z = seq_len * dim, hidden_dim, latent_dim
    r32 = lambda v: (v + 31) // 32 * 32  # noqa: E731
    f8 = fp8_layers(p, seq_len, dim, latent_dim, hidden_dim, n_enc, n_dec)
    shapes = {"condition_encoder.2": (H, H), "fc_mu": (2 * H, 2 * Z), "fc_logvar": (2 * H, 2 * Z)}
    for i in range(1, n_enc):
        shapes[f"encoder.{2 * i + 1}"] = (H, H)
    for i in range(n_dec):
        shapes[f"decoder.{2 * i}"] = (Z + H if i == 0 else H, I if i == n_dec - 1 else H)
    return {n: f8[n] for n, (k, o) in shapes.items()
            if n in f8 and r32(o) % 64 == 0 and (r32(o) >= 512 or r32(k) >= 512)}


def mx_dx(G, W, s):
    """dX = G·W of an f8b layer as the wide chain computes it (cvae_widechain.h gemm_mxb / mx_block):
    G (B, N) the bf16 gradient rows, W (N, K) the layer's weight, s its e4m3 weight scale.  The
    block-scaled MFMA's 32-value MX blocks (their lane / byte mapping measured on the GPU by
    scripts/ubench/mxscale.hip), in the gradient's feature order: within each 128-feature group,
    block (half, jj) = positions 16a + 8jj + i (a, i ranging) of the two chunks 2·half, 2·half + 1.
    Each block is scaled by 2^kb, kb = 134 − (biased fp32 exponent of max|block|) =
    7 − floor(log2 max|block|) (0 for an all-zero block, at most 126), rounded to e4m3 and unscaled in
    the product; W enters as e4m3(s·W)/s."""
    G = np.asarray(G, np.float32)
    B, N = G.shape
    Np = (N + 127) // 128 * 128
    Gp = np.zeros((B, Np), np.float32)
    Gp[:, :N] = G
    g7 = Gp.reshape(B, Np // 128, 2, 2, 2, 2, 8)  # (row, group, half, chunk, a, jj, i)
    amax = np.abs(g7).max(axis=(3, 4, 6), keepdims=True)
    eb = ((amax.view(np.uint32) >> 23) & 0xFF).astype(np.int64)
    kb = np.where(eb > 0, np.minimum(134 - eb, 126), 0).astype(np.float64)
    sc = np.exp2(kb).astype(np.float32)
    x8 = (e4m3(g7 * sc) / sc).reshape(B, Np)[:, :N]
    w8 = e4m3(np.asarray(W, np.float32) * s) / s
    return (x8.astype(np.float64) @ w8.astype(np.float64)).astype(np.float32)


def mx_dw(G, X):
    """dW = Gᵀ·X of a layer whose weight-gradient GEMM runs in e4m3 with MX scales along the batch
    (the wide fp8 dW, cvae_wgrad.h mx_dw_chunk; CVAE_FP8_DW=mx): G (B, N) and X (B, K) the bf16
    arena rows.  Every 32 consecutive batch rows of one feature are one MX block of the block-scaled
    MFMA (K = the batch: a 128-row chunk per instruction, block b = rows 32b..32b+31 of it); each
    block is scaled by 2^kb, kb = 134 − (biased fp32 exponent of max|block|) (0 for an all-zero
    block, at most 126), rounded to e4m3 and unscaled in the product — both operands alike."""
    def blocks(A):
        A = np.asarray(A, np.float32)
        B, F = A.shape
        Bp = (B + 31) // 32 * 32
        Ap = np.zeros((Bp, F), np.float32)
        Ap[:B] = A
        a3 = Ap.reshape(Bp // 32, 32, F)
        amax = np.abs(a3).max(axis=1, keepdims=True)
        eb = ((amax.view(np.uint32) >> 23) & 0xFF).astype(np.int64)
        kb = np.where(eb > 0, np.minimum(134 - eb, 126), 0).astype(np.float64)
        sc = np.exp2(kb).astype(np.float32)
        return (e4m3(a3 * sc) / sc).reshape(Bp, F)
    return (blocks(G).astype(np.float64).T @ blocks(X).astype(np.float64)).astype(np.float32)


def mxw_layers(p, n_enc=4, n_dec=4):
    """The layers whose dW the wide fp8 MX dW kernel computes in e4m3 (its 32 × 64 tiles: padded K a
    multiple of 64 — every layer but the K=2 condition layer); fc_mu / fc_logvar are one layer."""
    names = ["condition_encoder.2"] + [f"encoder.{2 * i + 1}" for i in range(n_enc)] + ["fc_mu", "fc_logvar"] \
        + [f"decoder.{2 * i}" for i in range(n_dec)]
    return {n for n in names if (p[n + ".weight"].shape[1] + 31) // 32 * 32 % 64 == 0}


def forward(p, x, eps, n_enc=4, n_dec=4, dt=np.float32, q=None, f8=None, q_layers=None):
    """x: (B,S,D) absolute trajectories.  Returns (recon, mu, logvar, h_c, cache).

    q: operand quantiser (``bf16`` emulates the bf16 kernel path exactly: GEMM operands and
    stored activations rounded, accumulation and recon/loss in fp32, loss target = q(x_rel)).
    f8: {layer name: scale} (``fp8_layers``) — those forward GEMMs run as e4m3 x e4m3 (CVAE_FP8).
    q_layers: the layers whose GEMM operands ``q`` rounds (default every layer) — attribution
    experiments: one layer rounded at a time (tests/test_attribution.py).
    """
    q = q or _ident
    f8 = f8 or {}

    def lin(x, p, name, q=q):  # the layer's fp8 scale, if it has one
        return _lin(x, p, name, q if q_layers is None or name in q_layers else _ident, f8.get(name))

    p = {k: v.astype(dt) for k, v in p.items()}
    x = x.astype(dt)
    B, S, D = x.shape
    start = x[:, 0, 1:3].copy()
    rel = x.copy()
    rel[:, :, 1:3] -= start[:, None, :]
    rel = q(rel)
    c = {"start": q(start), "rel": rel, "eps": eps.astype(dt), "q": q}
    a = rel.reshape(B, S * D)
    c["enc_in"] = [a]
    for i in range(n_enc):
        a = np.maximum(lin(a, p, f"encoder.{2 * i + 1}"), 0)
        c["enc_in"].append(a)
    h1 = np.maximum(lin(start, p, "condition_encoder.0"), 0)
    hc = np.maximum(lin(h1, p, "condition_encoder.2"), 0)
    c["hc1"], c["hc"] = h1, hc
    h = np.concatenate([a, hc], 1)
    c["h"] = h
    mu, lv = lin(h, p, "fc_mu"), lin(h, p, "fc_logvar")
    std = np.exp(dt(0.5) * lv)
    z = mu + c["eps"] * std
    c["std"] = std
    d = np.concatenate([z, hc], 1)
    c["dec_in"] = [d]
    for i in range(n_dec - 1):
        d = np.maximum(lin(d, p, f"decoder.{2 * i}"), 0)
        c["dec_in"].append(d)
    r = lin(d, p, f"decoder.{2 * (n_dec - 1)}").reshape(B, S, D)
    return r, mu, lv, hc, c


def losses(r, x_rel, mu, lv, w=(0.1, 0.1, 1.0, 1.0)):
    B, S, D = r.shape
    rec = np.mean((r - x_rel) ** 2)
    kld = -0.5 * np.mean(1 + lv - mu ** 2 - np.exp(lv))
    st = np.mean((r[:, 0, 1:3] - x_rel[:, 0, 1:3]) ** 2)
    tl = np.mean(r[:, 0, 0] ** 2) + np.mean(np.maximum(r[:, :-1, 0] - r[:, 1:, 0], 0))
    tot = w[0] * rec + w[1] * kld + w[2] * st + w[3] * tl
    return np.array([tot, rec, kld, st, tl])


def dloss_drecon(r, x_rel, w=(0.1, 0.1, 1.0, 1.0), B_norm=None):
    B, S, D = r.shape
    Bn = B if B_norm is None else B_norm
    g = w[0] * 2 * (r - x_rel) / (Bn * S * D)
    g[:, 0, 1:3] += w[2] * 2 * (r[:, 0, 1:3] - x_rel[:, 0, 1:3]) / (2 * Bn)
    g[:, 0, 0] += w[3] * 2 * r[:, 0, 0] / Bn
    m = (r[:, :-1, 0] > r[:, 1:, 0]).astype(r.dtype) * (w[3] / (Bn * (S - 1)))
    g[:, :-1, 0] += m
    g[:, 1:, 0] -= m
    return g


def backward(p, c, r, mu, lv, w=(0.1, 0.1, 1.0, 1.0), n_enc=4, n_dec=4, dt=np.float32, f8b=None, mxw=None,
             trace=None):
    """Gradients of the total loss w.r.t. every parameter (dict keyed like state_dict).

    With the cache of ``forward(..., q=bf16)`` every stored gradient G and every GEMM operand
    is rounded as the bf16 kernels round them (dz, the decoder's dh_c share, accumulations and
    the loss stay fp32).  f8b: {layer name: weight scale} (``fp8b_layers``) — those layers' dX
    GEMMs run in e4m3 with MX row-block scales (``mx_dx``; the wide chain's CVAE_FP8 form); their
    dW stays bf16 — unless the layer is in ``mxw`` (``mxw_layers``): then its dW is ``mx_dw``.
    trace: a dict that receives {layer name: (G, X)}, the rounded operands of each dW GEMM.
    """
    f8b = f8b or {}
    mxw = mxw or set()
    q = c.get("q", _ident)
    p = {k: v.astype(dt) for k, v in p.items()}
    B, S, D = r.shape
    Z = mu.shape[1]
    g = {}

    def lin_grads(name, G, X):
        G, X = q(G), q(X)
        if trace is not None:  # the operands of the layer's dW GEMM (gT, xT of the arena)
            trace[name] = (G, X)
        g[name + ".weight"] = mx_dw(G, X) if name in mxw else G.T @ X
        g[name + ".bias"] = G.sum(0)
        if name in f8b:
            return mx_dx(G, p[name + ".weight"], f8b[name])
        return G @ q(p[name + ".weight"])

    G = dloss_drecon(r, c["rel"], w).reshape(B, S * D)
    for i in reversed(range(n_dec)):
        dX = lin_grads(f"decoder.{2 * i}", G, c["dec_in"][i])
        if i > 0:
            G = dX * (c["dec_in"][i] > 0)
    dz, dhc2 = dX[:, :Z], dX[:, Z:]
    dmu = w[1] * mu / (B * Z) + dz
    dlv = w[1] * 0.5 * (np.exp(lv) - 1) / (B * Z) + dz * c["eps"] * 0.5 * c["std"]
    h = c["h"]
    dh = lin_grads("fc_mu", dmu, h) + lin_grads("fc_logvar", dlv, h)
    H = c["hc"].shape[1]
    G = dh[:, :H] * (c["enc_in"][n_enc] > 0)
    for i in reversed(range(n_enc)):
        dX = lin_grads(f"encoder.{2 * i + 1}", G, c["enc_in"][i])
        if i > 0:
            G = dX * (c["enc_in"][i] > 0)
    Gc = (dh[:, H:] + dhc2) * (c["hc"] > 0)
    Gc1 = lin_grads("condition_encoder.2", Gc, c["hc1"]) * (c["hc1"] > 0)
    lin_grads("condition_encoder.0", Gc1, c["start"])
    return g


def adam(p, g, m, v, step, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8):
    """torch ``_single_tensor_adam`` (amsgrad=False, wd=0) on float32 arrays, in place."""
    f = np.float32
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    step_size = f(lr / bc1)
    bc2s = f(bc2 ** 0.5)
    for k in p:
        gg = g[k].astype(f)
        m[k] = (m[k] + f(1 - b1) * (gg - m[k])).astype(f)           # lerp, weight < 0.5 branch
        v[k] = (v[k] * f(b2) + f(1 - b2) * gg * gg).astype(f)
        denom = (np.sqrt(v[k]) / bc2s + f(eps)).astype(f)
        p[k] = (p[k] + (-step_size) * m[k] / denom).astype(f)
    return p, m, v
