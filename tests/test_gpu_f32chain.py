"""The fp32 ring chain at the reference's own configuration (cvae_f32chain.h; Training_VAE.py:274-282:
seq_len 10, dim 3, latent 8, hidden 128, 4+4 layers, fp32; BASELINE configs[0]) against the generic
fp32 interpreter (CVAE_GENERIC=1) and the CPU oracle.  Needs the MI355X (-m gpu).

Tolerances: both kernels are exact fp32 MFMA chains that sum K in different orders, so against each
other losses rtol 1e-5 and gradients rel-L2 <= 1e-5; against the oracle (torch CPU fp32) the file-wide
fp32 tolerances of tests/test_hip_parity.py (losses 5e-5, gradients rel-L2 2e-4).  Repeated launches
are bit-identical (the K-split partials are reduced in a fixed order).

Every test runs on both row tilings of the chain (the `rows` fixture: CVAE_F32_ROWS=4, the
v_mfma_f32_4x4x1_16b_f32 form with K split over lane groups, and =16, the 16x16x4 form).
"""
import numpy as np
import pytest
import torch

from oracle import cvae_np
from oracle.cvae_oracle import OracleCVAE, oracle_loss, relative

pytestmark = pytest.mark.gpu
WD = dict(recon_weight=0.1, kld_weight=0.1, start_weight=1.0, time_weight=1.0)


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.fixture(scope="module")
def cvae():
    import cvae_amd
    assert torch.cuda.is_available()
    return cvae_amd


@pytest.fixture(params=[4, 16], ids=["rows4", "rows16"])
def rows(request, monkeypatch):
    """The chain's row tiling for every engine the test creates (CVAE_F32_ROWS at creation)."""
    monkeypatch.setenv("CVAE_F32_ROWS", str(request.param))
    return request.param


def _pair(cvae, monkeypatch, max_batch=256, seed=0, rows=None):
    """(f32-chain engine, generic-interpreter engine) bound to modules with the same init."""
    torch.manual_seed(seed)
    ref = OracleCVAE(10, 3, 8)
    m1 = cvae.ConditionalTrajectoryVAE(10, 3, 8)
    m1.load_state_dict(ref.state_dict())
    e1 = m1.attach(dtype="fp32", max_batch=max_batch, device="cuda:0", seed=7)
    monkeypatch.setenv("CVAE_GENERIC", "1")
    m2 = cvae.ConditionalTrajectoryVAE(10, 3, 8)
    m2.load_state_dict(ref.state_dict())
    e2 = m2.attach(dtype="fp32", max_batch=max_batch, device="cuda:0", seed=7)
    monkeypatch.delenv("CVAE_GENERIC")
    assert e1.train_kernel == "f32" and e2.train_kernel == "generic"
    if rows is not None:
        assert e1.chain_rows(1) == rows and e1.chain_rows(max_batch) == rows
    return ref, (m1, e1), (m2, e2)


def _data(n=300, seed=1):
    """Absolute trajectories like the sce1 data: a ~200 m start point plus metre-scale offsets."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 10, 3, generator=g) * 3
    x[:, :, 0] = torch.linspace(0, 9, 10)  # the time channel
    x[:, :, 1:] += torch.tensor([195.0, -12.0]) + torch.randn(n, 1, 2, generator=g) * 20
    return x


LAYERS = ["C0", "C1", "E0", "E1", "E2", "E3", "fc", "D0", "D1", "D2", "D3"]


@pytest.mark.parametrize("B", [38, 6])
def test_f32_chain_arena_matches_generic(cvae, monkeypatch, rows, B):
    """Every arena matrix the two chains write — each layer's input xT and pre-activation gradient
    gT, the dW kernel's operands — agrees (rows past the batch: gT zero in both)."""
    ref, (m1, e1), (m2, e2) = _pair(cvae, monkeypatch, rows=rows)
    x = _data().cuda()
    idx = torch.arange(B).cuda() * 3
    eps = torch.randn(B, 8, generator=torch.Generator().manual_seed(5))
    e1.forward_backward(x, idx=idx, eps=eps)
    e2.forward_backward(x, idx=idx, eps=eps)
    padded = (B + 31) // 32 * 32
    bad = []
    for l, name in enumerate(LAYERS):
        for which in ("x", "g"):
            a1 = e1.activation(l, which, padded).cpu().numpy()
            a2 = e2.activation(l, which, padded).cpu().numpy()
            r = rel_l2(a1[:B], a2[:B])
            print(f"{name} {which}T rel-L2 {r:.2e}")
            if not r < 1e-5:
                bad.append((name, which, r))
            if which == "g":
                assert not np.any(a1[B:]) and not np.any(a2[B:]), (name, "gT rows past the batch")
    assert not bad, bad


@pytest.mark.parametrize("B", [1, 6, 17, 32, 38, 64, 256])
def test_f32_chain_matches_generic(cvae, monkeypatch, rows, B):
    ref, (m1, e1), (m2, e2) = _pair(cvae, monkeypatch, rows=rows)
    x = _data().cuda()
    idx = torch.randperm(x.shape[0], generator=torch.Generator().manual_seed(B))[:B].cuda()
    eps = torch.randn(B, 8, generator=torch.Generator().manual_seed(100 + B))
    l1 = e1.forward_backward(x, idx=idx, eps=eps).cpu().numpy()
    l2 = e2.forward_backward(x, idx=idx, eps=eps).cpu().numpy()
    np.testing.assert_allclose(l1, l2, rtol=1e-5, atol=1e-8)
    g1, g2 = e1.grads.cpu().numpy(), e2.grads.cpu().numpy()
    for (o, n, _), k in zip(e1.tensors, cvae_np.param_keys()):
        assert rel_l2(g1[o:o + n], g2[o:o + n]) < 1e-5, (k, rel_l2(g1[o:o + n], g2[o:o + n]))


def test_f32_chain_philox_matches_generic(cvae, monkeypatch, rows):
    """In-kernel eps: the same Philox draws (seed, offset, global row) as the generic chain, also with
    a data-parallel row offset."""
    ref, (m1, e1), (m2, e2) = _pair(cvae, monkeypatch, rows=rows)
    x = _data(64).cuda()
    for row0 in (0, 96):
        l1 = e1.forward_backward(x, batch=38, row0=row0).cpu().numpy()
        l2 = e2.forward_backward(x, batch=38, row0=row0).cpu().numpy()
        np.testing.assert_allclose(l1, l2, rtol=1e-5, atol=1e-8)
        assert rel_l2(e1.grads.cpu(), e2.grads.cpu()) < 1e-5


@pytest.mark.parametrize("B", [6, 38, 200])
def test_f32_chain_vs_oracle(cvae, monkeypatch, rows, B):
    ref, (m1, e1), _ = _pair(cvae, monkeypatch, rows=rows)
    x = _data(B, seed=B)
    eps = torch.randn(B, 8, generator=torch.Generator().manual_seed(B))
    loss = e1.forward_backward(x, eps=eps).cpu().numpy()
    rel, start = relative(x)
    r, mu, lv, hc = ref(rel, start, eps)
    ls = oracle_loss(r, rel, mu, lv, hc, **WD)
    ls[0].backward()
    np.testing.assert_allclose(loss, [float(v) for v in ls], rtol=5e-5, atol=1e-7)
    g = {k: v.detach().cpu().numpy() for k, v in zip(m1.state_dict().keys(), e1.views(e1.grads))}
    for k, p in ref.named_parameters():
        assert rel_l2(g[k], p.grad.numpy()) < 2e-4, (k, rel_l2(g[k], p.grad.numpy()))


def test_f32_chain_training_steps_match_generic(cvae, monkeypatch, rows):
    """30 fused steps (dW ⊕ Adam behind each chain) over shuffled ragged batches stay within fp32
    reordering noise of the generic interpreter's run; the device step counters agree."""
    ref, (m1, e1), (m2, e2) = _pair(cvae, monkeypatch, rows=rows)
    x = _data(38).cuda()
    g = torch.Generator().manual_seed(3)
    for _ in range(15):
        perm = torch.randperm(38, generator=g).cuda()
        for lo, n in ((0, 32), (32, 6)):
            eps = torch.randn(n, 8, generator=g)
            e1.train_step(x, idx=perm[lo:lo + n], eps=eps)
            e2.train_step(x, idx=perm[lo:lo + n], eps=eps)
    torch.cuda.synchronize()
    assert torch.equal(e1.counters, e2.counters)
    assert rel_l2(e1.params.cpu(), e2.params.cpu()) < 1e-5
    np.testing.assert_allclose(e1.loss_accum.cpu().numpy(), e2.loss_accum.cpu().numpy(), rtol=1e-5)


def test_f32_chain_repeatable(cvae, monkeypatch, rows):
    """Repeated launches on one input give the same bits (deterministic K-split reductions, no
    data race in the ring or the images)."""
    _, (m1, e1), _ = _pair(cvae, monkeypatch, rows=rows)
    x = _data(64).cuda()
    eps = torch.randn(38, 8, generator=torch.Generator().manual_seed(9))
    l0 = e1.forward_backward(x, batch=38, eps=eps).clone()
    g0 = e1.grads.clone()
    for _ in range(100):
        l = e1.forward_backward(x, batch=38, eps=eps)
        assert torch.equal(l, l0) and torch.equal(e1.grads, g0)


def test_f32_chain_split_equals_fused(cvae, monkeypatch, rows):
    """fwd_bwd → Adam (the data-parallel route) equals the fused step bit for bit on the new chain."""
    _, (m1, e1), _ = _pair(cvae, monkeypatch, rows=rows)
    m3 = cvae.ConditionalTrajectoryVAE(10, 3, 8)
    m3.load_state_dict(m1.state_dict())
    e3 = m3.attach(dtype="fp32", max_batch=256, device="cuda:0", seed=7)
    assert e3.train_kernel == "f32" and e3.chain_rows(38) == rows
    x = _data(38).cuda()
    eps = torch.randn(38, 8, generator=torch.Generator().manual_seed(2))
    for _ in range(3):
        e1.train_step(x, eps=eps)
        e3.forward_backward(x, eps=eps)
        e3.adam_step(1.0)
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e3.params)
    assert torch.equal(e1.m, e3.m) and torch.equal(e1.v, e3.v)


@pytest.mark.parametrize("B", [32, 38, 6, 256])
def test_f32_dw_decode_equals_generic_tile_list(cvae, monkeypatch, rows, B):
    """The fp32 chain's dW ⊕ Adam launch decodes its tile and layer record from blockIdx
    (cvae_f32wgrad.h); CVAE_F32_DW=generic keeps the tile-list kernel.  Each tile is one
    independent wgrad_body, so the two equal each other bit for bit: gradients (split path), then
    params, moments, losses and counters after fused training steps (ragged last batch, Philox eps)."""
    torch.manual_seed(3)
    ref = OracleCVAE(10, 3, 8)
    engines = []
    for mode in (None, "generic"):
        if mode:
            monkeypatch.setenv("CVAE_F32_DW", mode)
        m = cvae.ConditionalTrajectoryVAE(10, 3, 8)
        m.load_state_dict(ref.state_dict())
        e = m.attach(dtype="fp32", max_batch=256, device="cuda:0", seed=11)
        monkeypatch.delenv("CVAE_F32_DW", raising=False)
        assert e.train_kernel == "f32" and e.chain_rows(B) == rows
        engines.append(e)
    e1, e2 = engines
    assert e1.dw_kernel == "f32" and e2.dw_kernel == "generic"
    x = _data(300, seed=B)
    xd1, xd2 = e1.as_input(x), e2.as_input(x)
    idx = torch.randperm(300, generator=torch.Generator().manual_seed(B))[:B].cuda()
    for e, xd in ((e1, xd1), (e2, xd2)):
        e.forward_backward(xd, idx=idx)
    torch.cuda.synchronize()
    assert torch.equal(e1.grads, e2.grads)
    for step in range(4):
        b = B if step < 3 else max(1, B // 3)  # a ragged last batch
        for e, xd in ((e1, xd1), (e2, xd2)):
            e.train_step(xd, idx=idx[:b])
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params)
    assert torch.equal(e1.m, e2.m) and torch.equal(e1.v, e2.v)
    assert torch.equal(e1.loss, e2.loss)
    assert torch.equal(e1.loss_accum, e2.loss_accum)
