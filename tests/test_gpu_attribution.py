"""Where the two parity outliers come from (VERDICT r05 "What's weak", parity): measured
attributions, printed by every run, with bounds at about 2x what was measured.  Needs the MI355X.

(a) fp8 at BASELINE cfg5: decoder.0.weight sits further from its emulation than every other
    gradient.  Its dW GEMM is gT(D0)ᵀ · xT(D0); the arena holds both operands as the kernels wrote
    them (cvae_read_activation), the emulation holds them as it rounded them (cvae_np.backward
    trace).  Swapping one operand at a time says which one carries the deviation, and counting the
    e4m3 flips of the decoder input [z ‖ h_c] (the twin the D0 forward GEMM multiplies) says how
    much of it is one-ulp rounding-boundary flips.  Measured (B = 64): the input is not it (xT(D0)
    within 3e-4, no e4m3 twin element differs); the gradient gT(D0) is (5.9 %).  The deviation grows
    through the decoder backward in jumps at the layers whose ReLU masks differ — 0.01-0.05 % of the
    hidden activations change sign between the kernel's e4m3 forward and the emulation's, and each
    flip moves one gradient element by its whole value — plus, with the reference's time weight,
    dL/drecon's monotonicity indicators (2.4 %).  decoder.0.weight shows it most because its input
    z has no sign structure to average it out.  Re-running the emulated backward on the kernel's own
    forward activations (masks and dW operands) takes decoder.0.weight from 0.056 to 0.018.
"""
import numpy as np
import pytest
import torch

from oracle import cvae_np
from oracle.cvae_oracle import OracleCVAE

pytestmark = pytest.mark.gpu
WIDE = dict(S=200, D=6, Z=512, n_enc=8, n_dec=8)


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.fixture(scope="module")
def cvae():
    import cvae_amd
    assert torch.cuda.is_available()
    return cvae_amd


@pytest.mark.parametrize("w_time", [1.0, 0.0])
def test_fp8_decoder0_weight_attribution(cvae, w_time):
    """With the reference weights the deviation is born in dL/drecon itself: its time channel
    carries the monotonicity term w_t/(B(S-1))·([r_s > r_{s+1}] - [r_{s-1} > r_s]) (Training_VAE.py
    :261-262), 30x the size of a recon-term entry at this shape, and a step function of the recon —
    wherever two neighbouring time values sit within the fp8 forward's noise of each other the
    indicator differs between kernel and emulation.  w_time = 0 removes the term: the deviation
    then falls to the bf16-dX level."""
    c = WIDE
    W = (0.1, 0.1, 1.0, w_time)
    B, S, D, Z, ne, nd = 64, c["S"], c["D"], c["Z"], c["n_enc"], c["n_dec"]
    torch.manual_seed(0)
    ref = OracleCVAE(S, D, Z, 128, ne, nd)
    m = cvae.ConditionalTrajectoryVAE(S, D, Z, 128, ne, nd)
    m.load_state_dict(ref.state_dict())
    eng = m.attach(dtype="fp8", max_batch=B, device="cuda:0")
    assert eng.train_kernel == "wide"
    x = torch.randn(B, S, D, generator=torch.Generator().manual_seed(1234)).to(torch.bfloat16).float()
    eps = torch.randn(B, Z, generator=torch.Generator().manual_seed(4321))
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    f8 = cvae_np.fp8_layers(p, S, D, Z, 128, ne, nd)
    f8b = cvae_np.fp8b_layers(p, S, D, Z, 128, ne, nd)
    r, mu, lv, hc, cc = cvae_np.forward(p, x.numpy(), eps.numpy(), n_enc=ne, n_dec=nd, q=cvae_np.bf16, f8=f8)
    tr = {}
    gw = cvae_np.backward(p, cc, r, mu, lv, w=W, n_enc=ne, n_dec=nd, f8b=f8b, trace=tr)
    eng.forward_backward(x, eps=eps, weights=W)
    g = {k: v.detach().cpu().numpy() for k, v in zip(m.state_dict().keys(), eng.views(eng.grads))}
    lD0 = 3 + ne  # state_dict layer order: C0, C1, E0..E7, fc, D0..
    Ge, Xe = tr["decoder.0"]
    Xk = eng.activation(lD0, "x", B).cpu().numpy()[:, :Z + 128]
    Gk = eng.activation(lD0, "g", B).cpu().numpy()[:, :128]
    e_full = rel_l2(g["decoder.0.weight"], gw["decoder.0.weight"])
    dw = lambda G, X: (G.astype(np.float64).T @ X.astype(np.float64))  # noqa: E731
    e_k = rel_l2(dw(Gk, Xk), gw["decoder.0.weight"])   # the kernel's own operands, fp64 sum
    e_x = rel_l2(dw(Ge, Xk), gw["decoder.0.weight"])   # only xT(D0) from the kernel
    e_g = rel_l2(dw(Gk, Xe), gw["decoder.0.weight"])   # only gT(D0) from the kernel
    z_e, h_e = Xe[:, :Z], Xe[:, Z:]
    z_k, h_k = Xk[:, :Z], Xk[:, Z:]
    f8_e, f8_k = cvae_np.e4m3(Xe), cvae_np.e4m3(Xk)
    flips = float(np.mean(f8_e != f8_k))
    print(f"decoder.0.weight vs emulation: {e_full:.4f} (kernel operands summed in fp64: {e_k:.4f}); "
          f"kernel xT(D0) alone {e_x:.4f}, kernel gT(D0) alone {e_g:.4f}")
    print(f"xT(D0) = [z ‖ h_c] vs emulation: z rel-L2 {rel_l2(z_k, z_e):.4f}, h_c {rel_l2(h_k, h_e):.4f}; "
          f"bf16 elements differing {np.mean(Xk != Xe):.3f}, e4m3 twin elements differing {flips:.3f}; "
          f"gT(D0) rel-L2 {rel_l2(Gk, Ge):.4f}")
    # the arena operands of every layer against the emulation's, in backward order
    order = [f"decoder.{2 * i}" for i in reversed(range(nd))] + ["fc_mu"] + \
            [f"encoder.{2 * i + 1}" for i in reversed(range(ne))] + ["condition_encoder.2", "condition_encoder.0"]
    index = {"condition_encoder.0": 0, "condition_encoder.2": 1, "fc_mu": 2 + ne}
    index.update({f"encoder.{2 * i + 1}": 2 + i for i in range(ne)})
    index.update({f"decoder.{2 * i}": 3 + ne + i for i in range(nd)})
    for name in order:
        G, X = tr[name]
        gk = eng.activation(index[name], "g", B).cpu().numpy()[:, :G.shape[1]]
        xk = eng.activation(index[name], "x", B).cpu().numpy()[:, :X.shape[1]]
        print(f"{name:20s} gT rel-L2 {rel_l2(gk, G):.4f}  xT rel-L2 {rel_l2(xk, X):.4f}  "
              f"weight grad {rel_l2(g[name + '.weight'], gw[name + '.weight']):.4f}")
    # the dW kernel itself is not the source: its result equals the fp64 product of its own operands
    assert abs(e_full - e_k) < 0.1 * e_full + 1e-3, (e_full, e_k)
    # nor the decoder input (the e4m3 twin the D0 forward multiplies): the kernel's xT(D0) with the
    # emulation's gT(D0) reproduces the emulation's gradient (measured 0.0003)
    assert e_x < 2e-3 and flips < 1e-3, (e_x, flips)
    g_d7 = rel_l2(eng.activation(3 + ne + nd - 1, "g", B).cpu().numpy()[:, :S * D], tr[f"decoder.{2 * (nd - 1)}"][0])
    print(f"w_time {w_time}: dL/drecon (gT of the last decoder layer) vs emulation {g_d7:.4f}")
    # ReLU mask flips: the sign pattern of every hidden activation, kernel against emulation
    H = 128
    xk = lambda l, n: eng.activation(l, "x", B).cpu().numpy()[:, :n]  # noqa: E731
    flip = {}
    for i in range(1, ne):
        flip[f"E{i - 1}"] = float(np.mean((xk(2 + i, H) > 0) != (cc["enc_in"][i] > 0)))
    for i in range(1, nd):
        flip[f"D{i - 1}"] = float(np.mean((xk(3 + ne + i, H) > 0) != (cc["dec_in"][i] > 0)))
    print("ReLU mask flips (fraction of elements):", {k: round(v, 5) for k, v in flip.items()})
    # the emulation's backward on the kernel's forward activations (its masks and dW operands): what is
    # left is the backward's own rounding (and, with w_time > 0, dL/drecon's indicators from the recon)
    c2 = dict(cc)
    c2["enc_in"] = [cc["enc_in"][0]] + [xk(2 + i, H) for i in range(1, ne)] + [xk(2 + ne, H)]
    c2["dec_in"] = [xk(3 + ne, Z + H)] + [xk(3 + ne + i, H) for i in range(1, nd)]
    c2["h"] = xk(2 + ne, 2 * H)
    c2["hc"] = c2["h"][:, H:]
    c2["hc1"] = xk(1, H)
    gw2 = cvae_np.backward(p, c2, r, mu, lv, w=W, n_enc=ne, n_dec=nd, f8b=f8b)
    e_kf = rel_l2(g["decoder.0.weight"], gw2["decoder.0.weight"])
    worst = max(cvae_np.param_keys(ne, nd), key=lambda k: rel_l2(g[k], gw2[k]))
    print(f"w_time {w_time}: decoder.0.weight vs the emulated backward on the kernel's activations {e_kf:.4f} "
          f"(against the plain emulation {e_full:.4f}); worst tensor there {worst} {rel_l2(g[worst], gw2[worst]):.4f}")
    # measured (w_time 1 / 0): decoder.0.weight 0.0564 / 0.0501 against the emulation; gT(D0) 0.0586 /
    # 0.0523; dL/drecon 0.0245 / 0.0069
    assert e_g > 0.8 * e_full and e_full < 0.13
    assert e_kf < 0.35 * e_full, (e_kf, e_full)
    # the backward pinned on the kernel's own forward: every gradient within 2x the measured worst
    # (decoder.0.weight 0.0183 with the time term, 0.0102 without) — against 0.13 for the plain
    # emulation (FP8_EMU_BOUNDS, tests/test_hip_parity.py), whose flips it no longer carries
    assert rel_l2(g[worst], gw2[worst]) < (0.04 if w_time > 0 else 0.025)
