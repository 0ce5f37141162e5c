"""BASELINE cfg4 on the MI355X: the scenario-class embedding (a build-side extension — the
reference conditions on the start point only, Training_VAE.py:132-137, :193, :214), checked
against the EXTENDED oracle (oracle/cvae_oracle.py OracleCVAE(n_classes, class_dim): e =
Embedding(class) concatenated beside h_c in both concats).  Parity unpinned vs the reference (it
has no such model); pinned to the oracle at the fp32 tolerances of test_hip_parity (losses rel <=
5e-5, grads rel-L2 <= 2e-4, params after 3 Adam steps rel-L2 <= 1e-4), bf16 vs fp32 at the bf16
ones.  All calls go through the C-ABI.
"""
import numpy as np
import pytest
import torch

from oracle.cvae_oracle import OracleCVAE, oracle_loss, relative

pytestmark = pytest.mark.gpu
WD = dict(recon_weight=0.1, kld_weight=0.1, start_weight=1.0, time_weight=1.0)
NC, E = 4, 16


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.fixture(scope="module")
def cvae():
    import cvae_amd
    assert torch.cuda.is_available()
    return cvae_amd


def _pair(cvae, S=10, D=3, dtype="fp32", max_batch=256, seed=0):
    torch.manual_seed(seed)
    ref = OracleCVAE(S, D, 8, n_classes=NC, class_dim=E)
    m = cvae.ConditionalTrajectoryVAE(S, D, 8, n_classes=NC, class_dim=E)
    m.load_state_dict(ref.state_dict())
    eng = m.attach(dtype=dtype, max_batch=max_batch, device="cuda:0")
    return ref, m, eng


@pytest.mark.parametrize("B", [1, 37, 256])
def test_cfg4_forward_loss_grads_vs_oracle(cvae, B):
    """Training step's forward, loss and every gradient (class_embedding.weight included) with an
    index gather over a 300-row dataset whose class ids are gathered by the same indices."""
    ref, m, eng = _pair(cvae)
    gen = torch.Generator().manual_seed(B)
    data = torch.randn(300, 10, 3, generator=gen) * 10
    cls_all = torch.randint(0, NC, (300,), generator=gen, dtype=torch.int32)
    idx = torch.randperm(300, generator=gen)[:B]
    eps = torch.randn(B, 8, generator=gen)
    loss = eng.forward_backward(data.cuda(), idx=idx.cuda(), eps=eps, classes=cls_all.cuda()).cpu().numpy()
    x = data[idx]
    rel, start = relative(x)
    r, mu, lv, hc = ref(rel, start, eps, cls_all[idx].long())
    ls = oracle_loss(r, rel, mu, lv, hc, **WD)
    ls[0].backward()
    np.testing.assert_allclose(loss, [float(v) for v in ls], rtol=5e-5, atol=1e-7)
    g = {k: v.detach().cpu().numpy() for k, v in zip(m.state_dict().keys(), eng.views(eng.grads))}
    for k, p in ref.named_parameters():
        assert rel_l2(g[k], p.grad.numpy()) < 2e-4, (k, rel_l2(g[k], p.grad.numpy()))
    # inference: forward outputs and class-conditioned decode
    r2, mu2, lv2, hc2 = eng.forward(x, eps=eps, classes=cls_all[idx])
    np.testing.assert_allclose(r2.cpu().numpy(), r.detach().numpy(), rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(mu2.cpu().numpy(), mu.detach().numpy(), rtol=1e-4, atol=2e-4)
    dec = m.decode(mu2, hc2, classes=cls_all[idx])
    with torch.no_grad():
        want = ref.decode(mu, hc, cls_all[idx].long())
    assert rel_l2(dec.cpu().numpy(), want.numpy()) < 1e-5


def test_cfg4_train_steps_vs_oracle_adam(cvae):
    """Three fused steps (row chain incl. the class-embedding step + dW ⊕ Adam over the 25 tensors)
    == three oracle steps with torch.optim.Adam."""
    from oracle.cvae_oracle import oracle_step
    ref, m, eng = _pair(cvae, seed=3)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(64, 10, 3, generator=gen) * 5
    cls = torch.randint(0, NC, (64,), generator=gen, dtype=torch.int32)
    for t in range(3):
        eps = torch.randn(64, 8, generator=gen)
        got = eng.train_step(x.cuda(), eps=eps, classes=cls.cuda()).cpu().numpy()
        rel, start = relative(x)
        opt.zero_grad()
        r, mu, lv, hc = ref(rel, start, eps, cls.long())
        ls = oracle_loss(r, rel, mu, lv, hc, **WD)
        ls[0].backward()
        opt.step()
        np.testing.assert_allclose(got, [float(v) for v in ls], rtol=5e-5, atol=1e-7)
    post = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    for k, v in ref.state_dict().items():
        assert rel_l2(post[k], v.numpy()) < 1e-4, (k, rel_l2(post[k], v.numpy()))


def test_cfg4_bf16_benchmark_shape(cvae):
    """cfg2's shape (S=100, D=6) with the class embedding, bf16 operands (the ring chain since round 3);
    losses within the bf16 tolerance of the fp32 oracle; 30 steps lower the ELBO; the split step
    equals the fused one bit for bit."""
    ref, m, eng = _pair(cvae, S=100, D=6, dtype="bf16", max_batch=512)
    m2 = cvae.ConditionalTrajectoryVAE(100, 6, 8, n_classes=NC, class_dim=E)
    m2.load_state_dict(ref.state_dict())
    e2 = m2.attach(dtype="bf16", max_batch=512, device="cuda:0")
    gen = torch.Generator().manual_seed(7)
    x = torch.randn(512, 100, 6, generator=gen).to(torch.bfloat16).float()
    cls = torch.randint(0, NC, (512,), generator=gen, dtype=torch.int32)
    eps = torch.randn(512, 8, generator=gen)
    loss = eng.forward_backward(x, eps=eps, classes=cls).cpu().numpy()
    rel, start = relative(x)
    r, mu, lv, hc = ref(rel, start, eps, cls.long())
    want = np.array([float(v) for v in oracle_loss(r, rel, mu, lv, hc, **WD)])
    np.testing.assert_allclose(loss, want, rtol=2e-2, atol=1e-5)
    xd, cd = eng.as_input(x), cls.cuda()
    eng.rng_offset, eng.step_count = 0, 0  # the loss check above began a step: both engines restart at 0
    for _ in range(3):
        eng.train_step(xd, classes=cd)
        e2.forward_backward(xd, classes=cd)
        e2.adam_step()
    torch.cuda.synchronize()
    assert torch.equal(eng.params, e2.params)
    first = eng.train_step(xd, classes=cd).clone()
    for _ in range(30):
        last = eng.train_step(xd, classes=cd)
    torch.cuda.synchronize()
    assert torch.isfinite(eng.params).all() and float(last[0]) < float(first[0])


def test_cfg4_train_loop_scenes(cvae, golden, tmp_path):
    """cvae_amd.train over several scene files (the class = the file index: Town04/Town05 scenes
    in one model) trains, saves 25 keys, and its class ids reach the kernel (a model trained on
    classes differs from one trained without)."""
    from cvae_amd.train import train
    x = golden("sce_fixed.npz")["sce1_x"].astype(np.float64)
    paths = []
    for i, scale in enumerate((1.0, 1.01, 0.99)):
        p = tmp_path / f"trajectory_sce{i + 1}_cond.npy"
        np.save(p, x * scale)
        paths.append(str(p))
    model, hist, _ = train([str(p) for p in paths], 10, 3, 8, batch_size=32, epochs=3, seed=0, log=None,
                           class_dim=8, model_save_path=str(tmp_path / "m.pth"))
    sd = torch.load(tmp_path / "m.pth", weights_only=True)
    assert len(sd) == 25 and tuple(sd["class_embedding.weight"].shape) == (3, 8)
    assert np.isfinite(hist["total_loss"]).all() and hist["total_loss"][-1] < hist["total_loss"][0]


def _ring_cls_pair(cvae, monkeypatch, B):
    torch.manual_seed(0)
    ref = OracleCVAE(100, 6, 8, n_classes=NC, class_dim=E)
    m1 = cvae.ConditionalTrajectoryVAE(100, 6, 8, n_classes=NC, class_dim=E)
    m1.load_state_dict(ref.state_dict())
    e1 = m1.attach(dtype="bf16", max_batch=B, device="cuda:0")
    monkeypatch.setenv("CVAE_GENERIC", "1")
    m2 = cvae.ConditionalTrajectoryVAE(100, 6, 8, n_classes=NC, class_dim=E)
    m2.load_state_dict(ref.state_dict())
    e2 = m2.attach(dtype="bf16", max_batch=B, device="cuda:0")
    monkeypatch.delenv("CVAE_GENERIC")
    return ref, m1, e1, m2, e2


@pytest.mark.parametrize("B", [37, 200, 1024])
def test_cfg4_ring_chain_vs_generic_and_oracle(cvae, monkeypatch, B):
    """BASELINE cfg4 at cfg2's shape runs the ring chain (train_kernel == "ring": the class
    embedding is one more K chunk of fc and part of the decoder input's padded K, its table the
    one-hot layer the generic dW kernel reduces).  Against the generic interpreter's bf16 chain
    (same rounding points, other fp32 summation orders): losses rtol 1e-3, every gradient —
    class_embedding.weight included — rel-L2 < 1e-2; against the fp32 extended oracle: losses at
    the bf16 tolerance (rtol 2e-2).  Ragged tile (37), gathered rows (200 of 300), B = 1024.
    Parity unpinned vs the reference, which has no class embedding."""
    ref, m1, e1, m2, e2 = _ring_cls_pair(cvae, monkeypatch, B)
    assert e1.train_kernel == "ring" and e2.train_kernel == "generic"
    gen = torch.Generator().manual_seed(B)
    n = max(B, 300)
    pool = torch.randn(n, 100, 6, generator=gen).to(torch.bfloat16)
    cls_all = torch.randint(0, NC, (n,), generator=gen, dtype=torch.int32)
    idx = torch.randperm(n, generator=gen)[:B]
    eps = torch.randn(B, 8, generator=gen)
    l1 = e1.forward_backward(pool.cuda(), idx=idx.cuda(), eps=eps, classes=cls_all.cuda()).cpu().numpy()
    l2 = e2.forward_backward(pool.cuda(), idx=idx.cuda(), eps=eps, classes=cls_all.cuda()).cpu().numpy()
    np.testing.assert_allclose(l1, l2, rtol=1e-3, atol=1e-6)
    g1 = {k: v.detach().cpu().numpy() for k, v in zip(m1.state_dict().keys(), e1.views(e1.grads))}
    g2 = {k: v.detach().cpu().numpy() for k, v in zip(m2.state_dict().keys(), e2.views(e2.grads))}
    assert "class_embedding.weight" in g1
    for k in g1:
        assert rel_l2(g1[k], g2[k]) < 1e-2, (k, rel_l2(g1[k], g2[k]))
    x = pool[idx].float()
    rel, start = relative(x)
    r, mu, lv, hc = ref(rel, start, eps, cls_all[idx].long())
    want = np.array([float(v) for v in oracle_loss(r, rel, mu, lv, hc, **WD)])
    np.testing.assert_allclose(l1, want, rtol=2e-2, atol=1e-5)


def test_cfg4_ring_training_split_equals_fused(cvae, monkeypatch):
    """Philox training on the cfg4 ring chain: the fused step (chain + generic dW ⊕ Adam) equals the
    split step (chain + dW, then Adam) bit for bit, a second engine replays it bit for bit, and 30
    steps lower the ELBO."""
    B = 256
    ref, m1, e1, m2, e2 = _ring_cls_pair(cvae, monkeypatch, B)
    m3 = cvae.ConditionalTrajectoryVAE(100, 6, 8, n_classes=NC, class_dim=E)
    m3.load_state_dict(ref.state_dict())
    e3 = m3.attach(dtype="bf16", max_batch=B, device="cuda:0")
    assert e3.train_kernel == "ring"
    gen = torch.Generator().manual_seed(9)
    xd = torch.randn(B, 100, 6, generator=gen).to("cuda", torch.bfloat16)
    cd = torch.randint(0, NC, (B,), generator=gen, dtype=torch.int32).cuda()
    first = e1.train_step(xd, classes=cd).clone()
    e3.forward_backward(xd, classes=cd)
    e3.adam_step()
    for _ in range(4):
        e1.train_step(xd, classes=cd)
        e3.forward_backward(xd, classes=cd)
        e3.adam_step()
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e3.params) and torch.equal(e1.m, e3.m) and torch.equal(e1.v, e3.v)
    for _ in range(25):
        last = e1.train_step(xd, classes=cd)
    torch.cuda.synchronize()
    assert torch.isfinite(e1.params).all() and float(last[0]) < float(first[0])


@pytest.mark.parametrize("E_", [4, 16, 24])
def test_cfg4_dw_decode_equals_generic_tile_list(cvae, monkeypatch, E_):
    """The ring chain's cfg4 form runs its dW ⊕ Adam with the tile and layer record decoded from
    blockIdx (wchain::clswgrad_kernel, class-dependent widths from two runtime arguments);
    CVAE_CLS_DW=generic keeps the tile-list kernel.  Same tiles, same order: gradients (split path),
    then params, moments and losses after fused steps (Philox eps, a ragged batch) bit for bit, for
    class_dim 4 / 16 / 24 (the padded widths do not move, the real ones and the offsets do)."""
    torch.manual_seed(5)
    ref = OracleCVAE(100, 6, 8, n_classes=NC, class_dim=E_)
    engines = []
    for mode in (None, "generic"):
        if mode:
            monkeypatch.setenv("CVAE_CLS_DW", mode)
        m = cvae.ConditionalTrajectoryVAE(100, 6, 8, n_classes=NC, class_dim=E_)
        m.load_state_dict(ref.state_dict())
        e = m.attach(dtype="bf16", max_batch=512, device="cuda:0", seed=3)
        monkeypatch.delenv("CVAE_CLS_DW", raising=False)
        assert e.train_kernel == "ring"
        engines.append(e)
    e1, e2 = engines
    assert e1.dw_kernel == "cls" and e2.dw_kernel == "generic"
    gen = torch.Generator().manual_seed(E_)
    data = torch.randn(600, 100, 6, generator=gen)
    cls_all = torch.randint(0, NC, (600,), generator=gen, dtype=torch.int32).cuda()
    x1, x2 = e1.as_input(data), e2.as_input(data)
    idx = torch.randperm(600, generator=gen)[:512].cuda()
    for e, x in ((e1, x1), (e2, x2)):
        e.forward_backward(x, idx=idx, classes=cls_all)
    torch.cuda.synchronize()
    assert torch.equal(e1.grads, e2.grads)
    for b in (512, 512, 300):
        for e, x in ((e1, x1), (e2, x2)):
            e.train_step(x, idx=idx[:b], classes=cls_all)
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params)
    assert torch.equal(e1.m, e2.m) and torch.equal(e1.v, e2.v)
    assert torch.equal(e1.loss, e2.loss)
