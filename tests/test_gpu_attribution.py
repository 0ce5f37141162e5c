"""Where the two parity outliers come from (VERDICT r05 "What's weak", parity): measured
attributions, printed by every run, with bounds at about 2x what was measured.  Needs the MI355X.

(a) fp8 at BASELINE cfg5: decoder.0.weight sits further from its emulation than every other
    gradient.  Its dW GEMM is gT(D0)ᵀ · xT(D0); the arena holds both operands as the kernels wrote
    them (cvae_read_activation), the emulation holds them as it rounded them (cvae_np.backward
    trace).  Swapping one operand at a time says which one carries the deviation, and counting the
    e4m3 flips of the decoder input [z ‖ h_c] (the twin the D0 forward GEMM multiplies) says how
    much of it is one-ulp rounding-boundary flips.
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


def test_fp8_decoder0_weight_attribution(cvae):
    c = WIDE
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
    gw = cvae_np.backward(p, cc, r, mu, lv, n_enc=ne, n_dec=nd, f8b=f8b, trace=tr)
    eng.forward_backward(x, eps=eps)
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
