"""HIP path vs the CPU oracle / reference goldens (needs the MI355X: -m gpu).

Tolerances (stated up front):
  fp32 path vs oracle: losses rel <= 1e-5 (2e-5 where a loss is a difference of
    large terms), grads rel-L2 <= 1e-4, params after Adam rel-L2 <= 1e-5.
  fp8 path (CVAE_FP8: e4m3 forward GEMMs, bf16 backward) vs the CPU emulation of its rounding
    points (oracle/cvae_np.py e4m3/fp8_layers): losses rel <= 5e-3, recon rel-L2 <= 1e-2, grads
    rel-L2 <= 1e-1 (median <= 2e-2: an e4m3 rounding flip moves an activation by 1/16); vs the fp32 reference the deviation is REPORTED (BASELINE cfg5: no parity
    claim) and only bounded loosely (losses rel <= 0.25).
  bf16 path (synthetic N(0,1), S=100 D=6): losses rel <= 2e-2, grads rel-L2 <= 5e-2 (1.2e-1 for
    the encoder L1 weight at B=64, where operand rounding alone gives 0.081); 200-step training
    curve within 2 % of the fp32 reference (10-step means; single steps 3 %).
All calls go through the C-ABI (libcvae_hip.so) via cvae_amd.
"""
import numpy as np
import pytest
import torch

from oracle import cvae_np
from oracle.cvae_oracle import OracleCVAE, oracle_loss, oracle_train, relative

pytestmark = pytest.mark.gpu
W = (0.1, 0.1, 1.0, 1.0)
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


def _model(cvae, S, D, Z, H=128, sd=None, dtype="fp32", max_batch=256, seed=0):
    m = cvae.ConditionalTrajectoryVAE(S, D, Z, H)
    if sd is not None:
        m.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()})
    eng = m.attach(dtype=dtype, max_batch=max_batch, device="cuda:0", seed=seed)
    return m, eng


def _grads(m, eng):
    return {k: v.detach().cpu().numpy() for k, v in zip(m.state_dict().keys(), eng.views(eng.grads))}


def test_forward_fixed_weights_zmu(cvae, golden):
    d = golden("sce_fixed.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w/")}
    m, eng = _model(cvae, 10, 3, 8, sd=sd)
    x = torch.from_numpy(d["sce1_x"])
    eps0 = torch.zeros(38, 8)
    recon, mu, lv, hc = eng.forward(x, eps=eps0)  # absolute x: transform in-kernel; z = mu
    np.testing.assert_allclose(mu.cpu().numpy(), d["sce1_mu"], rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(lv.cpu().numpy(), d["sce1_logvar"], rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(hc.cpu().numpy(), d["sce1_hc"], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(recon.cpu().numpy(), d["sce1_recon_zmu"], rtol=1e-4, atol=2e-4)
    ls = cvae.conditional_vae_loss(recon, relative(x)[0].cuda(), mu, lv, hc, **WD)
    np.testing.assert_allclose([float(v) for v in ls], d["sce1_losses_zmu"], rtol=1e-4, atol=1e-7)


def test_forward_relative_api_matches(cvae, golden):
    d = golden("sce_fixed.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w/")}
    m, eng = _model(cvae, 10, 3, 8, sd=sd)
    x = torch.from_numpy(d["sce1_x"])
    rel, start = relative(x)
    mu, lv, hc = m.encode(rel.cuda(), start.cuda())
    np.testing.assert_allclose(mu.cpu().numpy(), d["sce1_mu"], rtol=1e-4, atol=2e-4)
    r = m.decode(mu, hc)
    np.testing.assert_allclose(r.cpu().numpy(), d["sce1_recon_zmu"], rtol=1e-4, atol=2e-4)
    hc2 = m.condition_encoder(start.cuda())
    np.testing.assert_allclose(hc2.cpu().numpy(), d["sce1_hc"], rtol=1e-4, atol=1e-3)
    r2 = eng.decode(mu, start=start)
    np.testing.assert_allclose(r2.cpu().numpy(), d["sce1_recon_zmu"], rtol=1e-4, atol=2e-4)


def test_fwd_bwd_fixed_weights_grads(cvae, golden):
    d = golden("sce_fixed.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w/")}
    m, eng = _model(cvae, 10, 3, 8, sd=sd)
    assert eng.train_kernel == "f32"  # the reference's shape runs the fp32 ring chain (cvae_f32chain.h)
    x = torch.from_numpy(d["sce1_x"])
    loss = eng.forward_backward(x, eps=torch.from_numpy(d["sce1_eps"])).cpu().numpy()
    np.testing.assert_allclose(loss, d["sce1_losses_eps"], rtol=2e-5)
    g = _grads(m, eng)
    for k in cvae_np.param_keys():
        assert rel_l2(g[k], d["g/" + k]) < 1e-4, (k, rel_l2(g[k], d["g/" + k]))


def test_step1_h16_fused_step(cvae, golden):
    """H=16 exercises every padding path (H, 2H, Z+H, I all padded to 32)."""
    d = golden("step1_h16.npz")
    init = {k[5:]: d[k] for k in d.files if k.startswith("init/")}
    m, eng = _model(cvae, 10, 3, 8, H=16, sd=init)
    loss = eng.train_step(torch.from_numpy(d["x"]), eps=torch.from_numpy(d["eps"])).cpu().numpy()
    np.testing.assert_allclose(loss, d["losses"], rtol=2e-5)
    post = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    for k in cvae_np.param_keys():
        assert rel_l2(post[k], d["post/" + k]) < 1e-5, (k, rel_l2(post[k], d["post/" + k]))


def test_split_path_equals_fused(cvae, golden):
    """fwd_bwd → adam (the data-parallel path) == the fused wgrad+Adam kernel, bit for bit."""
    d = golden("step1_h16.npz")
    init = {k[5:]: d[k] for k in d.files if k.startswith("init/")}
    m1, e1 = _model(cvae, 10, 3, 8, H=16, sd=init)
    m2, e2 = _model(cvae, 10, 3, 8, H=16, sd=init)
    x, eps = torch.from_numpy(d["x"]), torch.from_numpy(d["eps"])
    for _ in range(3):
        e1.train_step(x, eps=eps)
        e2.forward_backward(x, eps=eps)
        e2.adam_step(1.0)
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params)
    assert torch.equal(e1.m, e2.m) and torch.equal(e1.v, e2.v)


def test_split_path_equals_fused_fast_kernels(cvae):
    """The data-parallel route at the benchmark's shape (bf16: fastwgrad<PM_GRAD> → param_kernel
    Adam) == the fused fastwgrad<PM_ADAM> step, bit for bit, and a grad_scale applied in the Adam
    kernel equals pre-scaling the gradient."""
    torch.manual_seed(0)
    ref = OracleCVAE(100, 6, 8)
    m1, e1 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=256)
    m2, e2 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=256)
    m3, e3 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=256)
    x = e1.as_input(torch.randn(256, 100, 6, generator=torch.Generator().manual_seed(5)))
    eps = torch.randn(256, 8, generator=torch.Generator().manual_seed(6)).cuda()
    for _ in range(3):
        e1.train_step(x, eps=eps)
        e2.forward_backward(x, eps=eps)
        e2.adam_step(1.0)
        e3.forward_backward(x, eps=eps)
        e3.grads.mul_(4.0)
        e3.adam_step(0.25)
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params)
    assert torch.equal(e1.m, e2.m) and torch.equal(e1.v, e2.v)
    assert torch.equal(e2.params, e3.params)  # ×4 then ×0.25: exact in fp32


def test_traj20_reference_train_loop(cvae, golden):
    """20 steps of Training_VAE.py's loop on sce1 (B=32, ragged 6-row batches) replayed on device."""
    d = golden("traj20_sce1.npz")
    x = golden("sce_fixed.npz")["sce1_x"]
    torch.manual_seed(int(d["seed"]))
    ref = OracleCVAE(10, 3, 8)
    m, eng = _model(cvae, 10, 3, 8, sd=ref.state_dict())
    assert eng.train_kernel == "f32"
    data = torch.from_numpy(x).cuda()
    order, eps_all, rows = d["order"], d["eps"], d["eps_rows"]
    o = 0
    losses = []
    for step, n in enumerate(rows):
        idx = torch.from_numpy(order[o:o + n]).cuda()
        eps = torch.from_numpy(eps_all[o:o + n])
        losses.append(eng.train_step(data, idx=idx, eps=eps).cpu().numpy().copy())
        o += n
    losses = np.array(losses)
    np.testing.assert_allclose(losses[:, 0], d["losses"][:, 0], rtol=1e-4)
    np.testing.assert_allclose(losses, d["losses"], rtol=2e-3, atol=1e-6)
    final = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    for k in cvae_np.param_keys():
        assert rel_l2(final[k], d["final/" + k]) < 1e-4, (k, rel_l2(final[k], d["final/" + k]))


def test_idx_gather_equals_pregathered(cvae):
    torch.manual_seed(0)
    m1, e1 = _model(cvae, 10, 3, 8)
    m2, e2 = _model(cvae, 10, 3, 8, sd=m1.state_dict())
    data = torch.randn(100, 10, 3) * 3
    idx = torch.randperm(100)[:40]
    eps = torch.randn(40, 8)
    l1 = e1.forward_backward(data.cuda(), idx=idx.cuda(), eps=eps)
    l2 = e2.forward_backward(data[idx].cuda(), eps=eps)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    assert torch.equal(e1.grads, e2.grads)


@pytest.mark.parametrize("B", [1, 17, 33, 38, 256])
def test_ragged_batches_vs_oracle(cvae, B):
    torch.manual_seed(B)
    ref = OracleCVAE(10, 3, 8)
    m, eng = _model(cvae, 10, 3, 8, sd=ref.state_dict())
    assert eng.train_kernel == "f32"
    x = torch.randn(B, 10, 3) * 10
    eps = torch.randn(B, 8)
    loss = eng.forward_backward(x, eps=eps).cpu().numpy()
    rel, start = relative(x)
    r, mu, lv, hc = ref(rel, start, eps)
    ls = oracle_loss(r, rel, mu, lv, hc, **WD)
    ls[0].backward()
    np.testing.assert_allclose(loss, [float(v) for v in ls], rtol=5e-5, atol=1e-7)
    g = _grads(m, eng)
    for k, p in ref.named_parameters():
        assert rel_l2(g[k], p.grad.numpy()) < 2e-4, (k, rel_l2(g[k], p.grad.numpy()))


def test_zero_weights_semantics(cvae):
    """start_weight/time_weight <= 0 skip those terms and report 0 (Training_VAE.py:246-264)."""
    torch.manual_seed(3)
    ref = OracleCVAE(10, 3, 8)
    m, eng = _model(cvae, 10, 3, 8, sd=ref.state_dict())
    x = torch.randn(20, 10, 3)
    eps = torch.randn(20, 8)
    w = (0.3, 0.2, 0.0, 0.0)
    loss = eng.forward_backward(x, eps=eps, weights=w).cpu().numpy()
    rel, start = relative(x)
    r, mu, lv, hc = ref(rel, start, eps)
    ls = oracle_loss(r, rel, mu, lv, hc, *w)
    ls[0].backward()
    np.testing.assert_allclose(loss, [float(v) for v in ls], rtol=5e-5, atol=1e-7)
    g = _grads(m, eng)
    for k, p in ref.named_parameters():
        assert rel_l2(g[k], p.grad.numpy()) < 2e-4, k


def _cfg2(cvae, dtype, B, seed=0):
    torch.manual_seed(seed)
    ref = OracleCVAE(100, 6, 8)
    m, eng = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype=dtype, max_batch=max(B, 32))
    x = torch.randn(B, 100, 6, generator=torch.Generator().manual_seed(1234))
    eps = torch.randn(B, 8, generator=torch.Generator().manual_seed(4321))
    return ref, m, eng, x, eps


# bf16 vs the fp32 reference: the CPU bf16 emulation (tests/golden-free, oracle/cvae_np.py q=bf16)
# shows rel-L2 up to 0.081 (encoder L1 weight, B=64) / 0.031 (B=1024) from operand rounding
# alone; the tolerances below bound that, and the emulation test above pins the kernel tightly.
# Loss terms: SURVEY §8c's ELBO tolerance (rel <= 1e-2); the emulation's own distance from fp32 is
# <= 3.5e-3 (KL and start terms) at B = 64 and 1024.
@pytest.mark.parametrize("dtype,B,ltol,gtol", [("fp32", 64, 2e-5, 1e-4), ("bf16", 64, 1e-2, 1.2e-1),
                                               ("bf16", 1024, 1e-2, 6e-2)])
def test_cfg2_shape_vs_oracle(cvae, golden, dtype, B, ltol, gtol):
    ref, m, eng, x, eps = _cfg2(cvae, dtype, B)
    if dtype == "bf16":
        x = x.to(torch.bfloat16).float()  # the bf16 path sees bf16 inputs; compare on the same data
    loss = eng.forward_backward(x, eps=eps).cpu().numpy()
    rel, start = relative(x)
    r, mu, lv, hc = ref(rel, start, eps)
    ls = oracle_loss(r, rel, mu, lv, hc, **WD)
    ls[0].backward()
    want = np.array([float(v) for v in ls])
    if dtype == "fp32" and B == 64:
        np.testing.assert_allclose(want, golden("cfg2_small.npz")["losses"], rtol=1e-6)
    np.testing.assert_allclose(loss, want, rtol=ltol, atol=1e-6)
    g = _grads(m, eng)
    for k, p in ref.named_parameters():
        assert rel_l2(g[k], p.grad.numpy()) < gtol, (k, rel_l2(g[k], p.grad.numpy()))


@pytest.mark.parametrize("B", [37, 1024])
def test_ring_chain_reconstruction_bf16_vs_oracle(cvae, B):
    """north_star: "reconstructions and ELBO match the reference CPU VAE within a stated fp
    tolerance" at the headline dtype — recon (Training_VAE.py:215), mu and logvar (:195-196) as the
    TRAINING step's ring chain computes them (cvae_tap_outputs: its own epilogue values, bf16
    operands and activations, fp32 accumulation), and the five loss terms (:240-267), on the same
    bf16-rounded inputs and eps.
    Against the fp32 oracle: recon rel-L2 <= 2e-2, ELBO terms rel <= 1e-2, mu / logvar
    rel-L2 <= 1e-2.  Against the CPU emulation of the chain's rounding points (cvae_np q=bf16):
    recon / mu / logvar rel-L2 <= 5e-3, losses rel <= 2e-3.  The tapped launch equals the untapped
    one bit for bit (the tap adds stores, not rounding points)."""
    ref, m, eng, x, eps = _cfg2(cvae, "bf16", B)
    assert eng.train_kernel == "ring"
    x = x.to(torch.bfloat16).float()
    recon, mu, lv = eng.forward_backward_outputs(x, eps=eps)
    loss = eng.loss.cpu().numpy()
    g_tap = eng.grads.clone()
    eng.forward_backward(x, eps=eps)
    torch.cuda.synchronize()
    assert np.array_equal(eng.loss.cpu().numpy(), loss) and torch.equal(eng.grads, g_tap)
    recon, mu, lv = recon.cpu().numpy(), mu.cpu().numpy(), lv.cpu().numpy()
    rel, start = relative(x)
    with torch.no_grad():
        r32, mu32, lv32, hc32 = ref(rel, start, eps)
        want = np.array([float(v) for v in oracle_loss(r32, rel, mu32, lv32, hc32, **WD)])
    dev = {"recon": rel_l2(recon, r32.numpy()), "mu": rel_l2(mu, mu32.numpy()), "logvar": rel_l2(lv, lv32.numpy())}
    lrel = np.abs(loss - want) / np.abs(want)
    print(f"bf16 ring chain B={B} vs fp32 oracle: {dev}, loss rel {lrel}")
    assert dev["recon"] <= 2e-2 and dev["mu"] <= 1e-2 and dev["logvar"] <= 1e-2, dev
    np.testing.assert_allclose(loss, want, rtol=1e-2, atol=1e-7)
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    re, mue, lve, _, c = cvae_np.forward(p, x.numpy(), eps.numpy(), q=cvae_np.bf16)
    de = {"recon": rel_l2(recon, re), "mu": rel_l2(mu, mue), "logvar": rel_l2(lv, lve)}
    print(f"  vs bf16 emulation: {de}")
    assert max(de.values()) <= 5e-3, de
    np.testing.assert_allclose(loss, cvae_np.losses(re, c["rel"], mue, lve), rtol=2e-3, atol=1e-7)


def test_armed_tap_is_consumed_by_fwd_bwd_only(cvae):
    """cvae_tap_outputs: while a tap is armed, a training call other than
    cvae_train_fwd_bwd fails and launches nothing (no write into buffers the caller may have freed);
    disarming with NULLs restores training, and the weights did not move in between."""
    import ctypes as C
    from cvae_amd._lib import lib
    ref, m, eng, x, eps = _cfg2(cvae, "bf16", 64)
    assert eng.train_kernel == "ring"
    x = x.to(torch.bfloat16).float()
    buf = torch.empty(64, 8, device="cuda:0")
    assert lib().cvae_tap_outputs(eng._h, None, C.c_void_p(buf.data_ptr()), None) == 0
    p0 = eng.params.clone()
    with pytest.raises(RuntimeError, match="armed"):
        eng.train_step(x, eps=eps)
    torch.cuda.synchronize()
    assert torch.equal(eng.params, p0)
    assert lib().cvae_tap_outputs(eng._h, None, None, None) == 0
    eng.train_step(x, eps=eps)
    torch.cuda.synchronize()
    assert not torch.equal(eng.params, p0)


def test_bf16_training_decreases_loss_full_size(cvae):
    """Size-independent property at the bench shape (B=1024, S=100, D=6): finite, decreasing ELBO."""
    torch.manual_seed(0)
    m, eng = _model(cvae, 100, 6, 8, dtype="bf16", max_batch=1024)
    x = torch.randn(1024, 100, 6, generator=torch.Generator().manual_seed(1234)).cuda()
    first = eng.train_step(x).clone()
    for _ in range(200):
        last = eng.train_step(x)
    torch.cuda.synchronize()
    assert torch.isfinite(eng.params).all()
    assert float(last[0]) < 0.7 * float(first[0])


def test_philox_forward_deterministic_per_offset(cvae):
    """Same (seed, offset) → bit-identical sampled forward; another offset → another draw.  (The
    distribution itself — mean, variance, KS, lag correlation over 2^20 draws — is checked by
    test_gpu_dp_autograd.py::test_philox_eps_statistics_and_determinism.)"""
    torch.manual_seed(0)
    m, eng = _model(cvae, 10, 3, 8, max_batch=4096, seed=123)
    x = torch.randn(4096, 10, 3).cuda()
    eng.rng_offset = 7
    r1, _, _, _ = eng.forward(x)
    eng.rng_offset = 7
    r2, _, _, _ = eng.forward(x)
    assert torch.equal(r1, r2)
    zs = []
    for off in range(2):
        eng.rng_offset = off
        rec, mu, lv, _ = eng.forward(x, outputs=("recon", "mu", "logvar"))
        zs.append(rec)
    assert not torch.equal(zs[0], zs[1])


def test_loss_kernel_matches_oracle(cvae):
    torch.manual_seed(5)
    B, S, D, Z = 70, 12, 4, 6
    r = torch.randn(B, S, D)
    x = torch.randn(B, S, D)
    mu, lv = torch.randn(B, Z), torch.randn(B, Z) * 0.5
    got = cvae.conditional_vae_loss(r.cuda(), x.cuda(), mu.cuda(), lv.cuda(), None, 0.2, 0.3, 0.7, 0.9)
    want = oracle_loss(r, x, mu, lv, None, 0.2, 0.3, 0.7, 0.9)
    np.testing.assert_allclose([float(v) for v in got], [float(v) for v in want], rtol=2e-5)


def test_generate_absolute(cvae):
    torch.manual_seed(0)
    m, eng = _model(cvae, 10, 3, 8)
    st = torch.tensor([[150.0, -10.0], [10.0, 20.0]])
    z = torch.randn(2, 8)
    rel, ab = m.generate(st, z=z.cuda())
    np.testing.assert_allclose((ab - rel)[:, :, 1:3].cpu().numpy(), st[:, None, :].expand(2, 10, 2).numpy(),
                               rtol=1e-6, atol=1e-4)


def test_load_model_and_generate_trajectory_matches_reference(cvae, golden, tmp_path):
    """Tools.py:18-65 drop-in: the reference function's own outputs on the shipped sce1 checkpoint
    (generate_sce1.npz, made by tests/golden/make_generate_goldens.py) from the same seeds —
    same z draw from the global CPU generator, same absolute trajectory (fp32 path)."""
    from cvae_amd import generate_trajectories, load_model_and_generate_trajectory
    w = golden("sce_fixed.npz")
    g = golden("generate_sce1.npz")
    path = tmp_path / "vae_offset_sce1_cond_ld8_epoch3000.pth"
    torch.save({k[2:]: torch.from_numpy(w[k]) for k in w.files if k.startswith("w/")}, path)
    for s, (sx, sy), want in zip(g["seeds"], g["starts"], g["traj"]):
        torch.manual_seed(int(s))
        got = load_model_and_generate_trajectory(str(path), float(sx), float(sy), seq_len=10, dim=3, latent_dim=8)
        assert got.shape == (10, 3)
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=2e-4)
    allg = generate_trajectories(str(path), g["starts"], seq_len=10, dim=3, latent_dim=8, z=torch.from_numpy(g["z"]))
    np.testing.assert_allclose(allg, g["traj"], rtol=1e-5, atol=2e-4)


@pytest.mark.parametrize("B", [64, 1024])
def test_bf16_path_matches_bf16_emulation(cvae, B):
    """The bf16 kernels against an exact CPU emulation of their rounding points
    (oracle/cvae_np.py forward/backward with q=bf16): this pins the bf16 path tightly, while
    test_cfg2_shape_vs_oracle bounds its distance from the fp32 reference."""
    ref, m, eng, x, eps = _cfg2(cvae, "bf16", B)
    x = x.to(torch.bfloat16).float()
    loss = eng.forward_backward(x, eps=eps).cpu().numpy()
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    r, mu, lv, hc, c = cvae_np.forward(p, x.numpy(), eps.numpy(), q=cvae_np.bf16)
    want = cvae_np.losses(r, c["rel"], mu, lv)
    np.testing.assert_allclose(loss, want, rtol=2e-3, atol=1e-6)
    gw = cvae_np.backward(p, c, r, mu, lv)
    g = _grads(m, eng)
    for k in cvae_np.param_keys():
        assert rel_l2(g[k], gw[k]) < 2e-2, (k, rel_l2(g[k], gw[k]))


def test_train_loop_end_to_end_traj20(cvae, golden, tmp_path):
    """cvae_amd.train (the Training_VAE.py __main__ loop) on device vs the reference's seeded run.

    Same seed → same init, DataLoader order and host eps stream; epoch means of the reference's
    per-step losses (:366-373) and its final parameters after 20 Adam steps.
    """
    from cvae_amd.train import LOSS_KEYS, train
    d = golden("traj20_sce1.npz")
    x = golden("sce_fixed.npz")["sce1_x"]
    model, hist, _ = train(x, 10, 3, 8, batch_size=int(d["batch_size"]), epochs=10, weights=W,
                           seed=int(d["seed"]), eps="host", log=None, dtype="fp32",
                           model_save_path=str(tmp_path / "m.pth"))
    steps = d["losses"]
    want = np.array([(steps[2 * e] * 32 + steps[2 * e + 1] * 6) / 38 for e in range(10)])
    got = np.array([hist[k] for k in LOSS_KEYS]).T
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=1e-4)
    np.testing.assert_allclose(got, want, rtol=2e-3, atol=1e-6)
    sd = torch.load(tmp_path / "m.pth", weights_only=True)
    assert len(sd) == 24
    for k in cvae_np.param_keys():
        assert rel_l2(sd[k].numpy(), d["final/" + k]) < 1e-4, k


@pytest.mark.parametrize("dtype,S,D,eps", [("fp32", 10, 3, "host"), ("bf16", 100, 6, "philox")])
def test_train_epoch_chunks_bit_equal(cvae, tmp_path, dtype, S, D, eps):
    """train()'s fused epoch loop on device: chunks of 1 and 3 epochs per C call (the next chunk's
    host draws and pinned non-blocking uploads queued behind the running chunk; a cut-short last
    chunk) give the same loss history and parameters, bit for bit, as all 7 epochs in one call."""
    from cvae_amd.train import LOSS_KEYS, train
    x = np.random.default_rng(5).normal(size=(300, S, D)).astype(np.float32)
    out = []
    for epc in (64, 3, 1):
        torch.manual_seed(11)
        m, hist, _ = train(x, S, D, 8, batch_size=64, epochs=7, weights=W, seed=11, eps=eps, log=None,
                           dtype=dtype, epochs_per_call=epc, model_save_path=str(tmp_path / f"m{epc}.pth"))
        out.append((np.array([hist[k] for k in LOSS_KEYS]), torch.load(tmp_path / f"m{epc}.pth", weights_only=True)))
    for h, sd in out[1:]:
        np.testing.assert_array_equal(h, out[0][0])
        for k, v in sd.items():
            assert torch.equal(v, out[0][1][k]), k


def test_train_steps_equals_repeated_train_step(cvae):
    """cvae_train_steps (one C call for n steps) == n train_step calls, bit for bit (bf16 fast
    chain and fp32 generic chain), with per-step rows from idx and Philox eps offsets."""
    for dtype, S, D in (("bf16", 100, 6), ("fp32", 10, 3)):
        torch.manual_seed(0)
        ref = OracleCVAE(S, D, 8)
        m1, e1 = _model(cvae, S, D, 8, sd=ref.state_dict(), dtype=dtype, max_batch=64)
        m2, e2 = _model(cvae, S, D, 8, sd=ref.state_dict(), dtype=dtype, max_batch=64)
        data = torch.randn(300, S, D).cuda()
        idx = torch.randint(0, 300, (3 * 64,)).cuda()
        for i in range(3):
            e1.train_step(data, idx=idx[i * 64:(i + 1) * 64])
        e2.train_steps(data, 3, idx=idx, batch=64)
        torch.cuda.synchronize()
        assert torch.equal(e1.params, e2.params), dtype
        assert torch.equal(e1.loss, e2.loss) and torch.equal(e1.loss_accum, e2.loss_accum), dtype


def _bf16_run(cvae, sd, x, idx_list, monkeypatch=None, env=None):
    if monkeypatch is not None:
        if env:
            monkeypatch.setenv(*env)
        else:
            monkeypatch.delenv("CVAE_GENERIC", raising=False)
    m, e = _model(cvae, 100, 6, 8, sd=sd, dtype="bf16", max_batch=200)
    if monkeypatch is not None and env:
        monkeypatch.delenv(env[0])
    losses = []
    for idx in idx_list:
        e.train_step(x, idx=idx, eps=torch.zeros(idx.numel(), 8).cuda() + 0.25)
        losses.append(e.loss.clone())
    torch.cuda.synchronize()
    return e, torch.stack(losses)


def test_fast_and_generic_kernels_agree(cvae, monkeypatch):
    """The specialised bf16 kernels (fastchain + fastwgrad) and the generic interpreter
    (CVAE_GENERIC=1 at handle creation) compute the same training steps, up to fp32 summation
    order: losses and parameters after 3 steps, ragged batch included."""
    torch.manual_seed(0)
    ref = OracleCVAE(100, 6, 8)
    x = torch.randn(300, 100, 6).to("cuda", torch.bfloat16)
    idxs = [torch.randint(0, 300, (B,), generator=torch.Generator().manual_seed(B)).cuda() for B in (200, 77, 160)]
    ef, lf = _bf16_run(cvae, ref.state_dict(), x, idxs, monkeypatch)
    eg, lg = _bf16_run(cvae, ref.state_dict(), x, idxs, monkeypatch, ("CVAE_GENERIC", "1"))
    np.testing.assert_allclose(lf.cpu().numpy(), lg.cpu().numpy(), rtol=2e-3, atol=1e-6)
    dp = (ef.params - eg.params).norm() / (ef.params - torch.cat([p.detach().flatten() for p in ref.parameters()]).cuda()).norm()
    assert float(dp) < 2e-2, float(dp)  # relative to the 3-step update


def _ring_pair(cvae, monkeypatch, B, seed=0):
    """Two bf16 engines of the reference architecture (S=100, D=6) on the same weights: the
    single-ring chain (the default, cvae_widechain.h small-latent form) and fastchain_kernel
    (CVAE_RING=0 at creation)."""
    torch.manual_seed(seed)
    ref = OracleCVAE(100, 6, 8)
    monkeypatch.delenv("CVAE_GENERIC", raising=False)
    monkeypatch.delenv("CVAE_RING", raising=False)
    m1, e1 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=max(B, 32))
    monkeypatch.setenv("CVAE_RING", "0")
    m2, e2 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=max(B, 32))
    monkeypatch.delenv("CVAE_RING")
    assert e1.train_kernel == "ring" and e2.train_kernel == "fast"
    return ref, m1, e1, m2, e2


@pytest.mark.parametrize("B", [37, 200, 1024])
def test_ring_chain_matches_fast_and_emulation(cvae, monkeypatch, B):
    """The ring chain (one weight stream per wave across every step; fc split over the waves by K)
    against fastchain_kernel (same rounding points; fp32 summation order of fc aside) and against
    the CPU emulation of those rounding points: ragged last tile (B=37), a gathered batch (B=200
    rows of 300 by index), the benchmark batch (B=1024)."""
    ref, m1, e1, m2, e2 = _ring_pair(cvae, monkeypatch, B)
    pool = torch.randn(max(B, 300), 100, 6, generator=torch.Generator().manual_seed(B)).to(torch.bfloat16)
    idx = torch.randperm(pool.shape[0], generator=torch.Generator().manual_seed(3))[:B]
    eps = torch.randn(B, 8, generator=torch.Generator().manual_seed(4321))
    l1 = e1.forward_backward(pool.cuda(), idx=idx.cuda(), eps=eps).cpu().numpy()
    l2 = e2.forward_backward(pool.cuda(), idx=idx.cuda(), eps=eps).cpu().numpy()
    np.testing.assert_allclose(l1, l2, rtol=1e-3, atol=1e-6)
    g1, g2 = _grads(m1, e1), _grads(m2, e2)
    for k in g1:
        assert rel_l2(g1[k], g2[k]) < 1e-2, (k, rel_l2(g1[k], g2[k]))
    x = pool[idx].float()
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    r, mu, lv, hc, c = cvae_np.forward(p, x.numpy(), eps.numpy(), q=cvae_np.bf16)
    np.testing.assert_allclose(l1, cvae_np.losses(r, c["rel"], mu, lv), rtol=2e-3, atol=1e-6)
    ge = cvae_np.backward(p, c, r, mu, lv)
    for k in cvae_np.param_keys():
        assert rel_l2(g1[k], ge[k]) < 2e-2, (k, rel_l2(g1[k], ge[k]))


@pytest.mark.parametrize("B", [37, 1024])
def test_ring_chain_fp32_rows_relative_transform(cvae, monkeypatch, B):
    """The ring chain on fp32 rows (CVAE_X_F32: what the train loop hands it — real data with
    ~200 m absolute coordinates): the start point is subtracted in fp32 and the offsets rounded to
    bf16 once, as the generic interpreter does (CVAE_GENERIC=1).  Same rounding points: losses
    rtol 1e-3, gradients rel-L2 < 1e-2 (fp32 summation orders differ); against bf16 rows of the same
    data the relative offsets differ (rounded absolute coordinates), so the fp32 path is closer to
    the fp32 oracle."""
    torch.manual_seed(0)
    ref = OracleCVAE(100, 6, 8)
    monkeypatch.delenv("CVAE_GENERIC", raising=False)
    m1, e1 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=max(B, 32))
    monkeypatch.setenv("CVAE_GENERIC", "1")
    m2, e2 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=max(B, 32))
    monkeypatch.delenv("CVAE_GENERIC")
    assert e1.train_kernel == "ring" and e2.train_kernel == "generic"
    gen = torch.Generator().manual_seed(B)
    x = torch.randn(B, 100, 6, generator=gen)
    x[:, :, 1] += 180.0 + 40.0 * torch.rand(B, 1, generator=gen)   # absolute world coordinates
    x[:, :, 2] -= 150.0 + 40.0 * torch.rand(B, 1, generator=gen)
    eps = torch.randn(B, 8, generator=gen)
    for e in (e1, e2):
        e.keep_f32 = True
    xd = e1.as_input(x, keep_f32=True)
    assert xd.dtype == torch.float32
    l1 = e1.forward_backward(xd, eps=eps).cpu().numpy()
    l2 = e2.forward_backward(xd, eps=eps).cpu().numpy()
    np.testing.assert_allclose(l1, l2, rtol=1e-3, atol=1e-6)
    g1, g2 = _grads(m1, e1), _grads(m2, e2)
    for k in g1:
        assert rel_l2(g1[k], g2[k]) < 1e-2, (k, rel_l2(g1[k], g2[k]))
    rel, start = relative(x)
    r, mu, lv, hc = ref(rel, start, eps)
    want = np.array([float(v) for v in oracle_loss(r, rel, mu, lv, hc, 0.1, 0.1, 1.0, 1.0)])
    lb = e1.forward_backward(e1.as_input(x.to(torch.bfloat16)), eps=eps).cpu().numpy()
    assert np.abs(l1 - want).sum() < np.abs(lb - want).sum(), (l1, lb, want)


@pytest.mark.parametrize("kind", ["ring", "wide_bf16", "wide_fp8"])
def test_chain_row_formats_bit_equal(cvae, kind):
    """fp32 rows and bf16 rows run different instances of the chain (bf16 rows: the fp32-row loads
    compiled out, wide_body's XB).  On bf16-representable data with absolute coordinates they give
    the same bits: the fp32 form subtracts the start point in fp32 and rounds once, which is what
    the bf16 form computes from the same values.  With and without a row gather (idx), and with a
    ragged last row tile (B = 77)."""
    B, N = 77, 200
    if kind == "ring":
        torch.manual_seed(0)
        _, eng = _model(cvae, 100, 6, 8, dtype="bf16", max_batch=N)
        S, D, Z = 100, 6, 8
    else:
        _, _, eng, _, _ = _wide(cvae, kind[5:], N)
        S, D, Z = WIDE["S"], WIDE["D"], WIDE["Z"]
    assert eng.train_kernel == ("ring" if kind == "ring" else "wide")
    gen = torch.Generator().manual_seed(7)
    x = torch.randn(N, S, D, generator=gen)
    x[:, :, 1] += 180.0 + 40.0 * torch.rand(N, 1, generator=gen)   # absolute world coordinates
    x[:, :, 2] -= 150.0 + 40.0 * torch.rand(N, 1, generator=gen)
    x = x.to(torch.bfloat16)
    eps = torch.randn(B, Z, generator=gen)
    idx = torch.randperm(N, generator=gen)[:B]
    eng.keep_f32 = True
    x32, x16 = x.float().cuda(), x.cuda()
    for ix in (None, idx):
        out = []
        for xx in (x32, x16):
            assert eng._xflags(eng.as_input(xx, keep_f32=True)) == (1 if xx.dtype == torch.float32 else 0)
            l = eng.forward_backward(xx if ix is not None else xx[:B], idx=ix, eps=eps, batch=B).clone()
            out.append((l, eng.grads.clone()))
        assert torch.equal(out[0][0], out[1][0]), (ix is not None, out[0][0], out[1][0])
        assert torch.equal(out[0][1], out[1][1]), (ix is not None, (out[0][1] - out[1][1]).abs().max())


def test_ring_chain_philox_training_and_determinism(cvae, monkeypatch):
    """In-kernel Philox eps keyed by the global row: the ring chain draws fastchain's noise (same
    losses up to summation order); five training steps (device counters, dW ⊕ Adam behind each
    chain) stay within the bf16 summation-order distance of the fastchain run; a second ring
    engine replays the first bit for bit; the DP split path (row chain + dW without Adam, then
    Adam) equals the fused ring step bit for bit."""
    B = 160
    ref, m1, e1, m2, e2 = _ring_pair(cvae, monkeypatch, B)
    xd = torch.randn(B, 100, 6, generator=torch.Generator().manual_seed(5)).to("cuda", torch.bfloat16)
    l1 = e1.forward_backward(xd, row0=320).cpu().numpy()
    l2 = e2.forward_backward(xd, row0=320).cpu().numpy()
    np.testing.assert_allclose(l1, l2, rtol=1e-3, atol=1e-6)
    p0 = e1.params.clone()
    for _ in range(5):
        e1.train_step(xd)
        e2.train_step(xd)
    torch.cuda.synchronize()
    np.testing.assert_allclose(e1.loss.cpu().numpy(), e2.loss.cpu().numpy(), rtol=3e-3, atol=1e-6)
    dp = (e1.params - e2.params).norm() / (e1.params - p0).norm()
    assert float(dp) < 2e-2, float(dp)
    monkeypatch.setenv("CVAE_RING", "1")
    m3, e3 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=B)
    m4, e4 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=B)
    monkeypatch.delenv("CVAE_RING")
    assert e3.train_kernel == "ring" and e4.train_kernel == "ring"
    e3.forward_backward(xd, row0=320)
    e4.forward_backward(xd, row0=320)
    for _ in range(5):
        e3.train_step(xd)
        e4.forward_backward(xd)
        e4.adam_step(1.0)
    torch.cuda.synchronize()
    assert torch.equal(e3.params, e1.params) and torch.equal(e3.loss, e1.loss)
    assert torch.equal(e3.params, e4.params) and torch.equal(e3.m, e4.m) and torch.equal(e3.v, e4.v)


@pytest.mark.parametrize("ring", ["0", "1"])
def test_reference_chain_repeatable(cvae, monkeypatch, ring):
    """fastchain_kernel (default) and the ring chain (CVAE_RING=1) at the benchmark batch: eight
    forward_backward calls on the same input and eps give bit-equal losses and gradients."""
    torch.manual_seed(0)
    ref = OracleCVAE(100, 6, 8)
    monkeypatch.setenv("CVAE_RING", ring)
    m, e = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=1024)
    monkeypatch.delenv("CVAE_RING")
    assert e.train_kernel == ("ring" if ring == "1" else "fast")
    x = torch.randn(1024, 100, 6, generator=torch.Generator().manual_seed(11)).to("cuda", torch.bfloat16)
    eps = torch.randn(1024, 8, generator=torch.Generator().manual_seed(12))
    l0 = e.forward_backward(x, eps=eps).clone()
    g0 = e.grads.clone()
    for _ in range(7):
        assert torch.equal(e.forward_backward(x, eps=eps), l0) and torch.equal(e.grads, g0)


def test_misaligned_input_runs_generic_chain(cvae):
    """x whose data pointer is not 16-B aligned takes the generic row chain (the fast chain loads
    16-B vectors) with the fast dW kernel behind it; the result matches the aligned run."""
    torch.manual_seed(0)
    ref = OracleCVAE(100, 6, 8)
    B = 64
    xa = torch.randn(B, 100, 6).to("cuda", torch.bfloat16)
    flat = torch.empty(B * 600 + 1, dtype=torch.bfloat16, device="cuda")
    flat[1:] = xa.flatten()
    xm = flat[1:].view(B, 100, 6)
    assert xm.data_ptr() % 16 != 0 and xm.is_contiguous()
    m1, e1 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=B)
    m2, e2 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=B)
    eps = torch.randn(B, 8).cuda()
    for _ in range(2):
        e1.train_step(xa, eps=eps)
        e2.train_step(xm, eps=eps)
    torch.cuda.synchronize()
    np.testing.assert_allclose(e1.loss.cpu().numpy(), e2.loss.cpu().numpy(), rtol=2e-3, atol=1e-6)
    assert float((e1.params - e2.params).norm() / e1.params.norm()) < 1e-3


# ---- BASELINE cfg5 shape: latent 512, 8 + 8 layers, seq_len 200 (bf16 operands, and the fp8
# forward-GEMM variant at the end of this file).  The generic row chain runs it with 8-row tiles (bf16) or 4-row tiles
# (fp32): the tile state does not fit 16 rows in 160 KiB of LDS at this width.
WIDE = dict(S=200, D=6, Z=512, n_enc=8, n_dec=8)


def _wide(cvae, dtype, B, seed=0):
    torch.manual_seed(seed)
    ref = OracleCVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    m = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    m.load_state_dict(ref.state_dict())
    eng = m.attach(dtype=dtype, max_batch=max(B, 32), device="cuda:0")
    x = torch.randn(B, WIDE["S"], WIDE["D"], generator=torch.Generator().manual_seed(1234))
    eps = torch.randn(B, WIDE["Z"], generator=torch.Generator().manual_seed(4321))
    return ref, m, eng, x, eps


def _oracle_grads(ref, x, eps):
    rel, start = relative(x)
    r, mu, lv, hc = ref(rel, start, eps)
    ls = oracle_loss(r, rel, mu, lv, hc, **WD)
    ls[0].backward()
    return np.array([float(v.detach()) for v in ls]), {k: p.grad.numpy() for k, p in ref.named_parameters()}


@pytest.mark.parametrize("B", [37, 128])
def test_wide_cfg5_fp32_vs_oracle(cvae, B):
    ref, m, eng, x, eps = _wide(cvae, "fp32", B)
    assert list(m.state_dict().keys()) == list(ref.state_dict().keys())
    loss = eng.forward_backward(x, eps=eps).cpu().numpy()
    want, gw = _oracle_grads(ref, x, eps)
    np.testing.assert_allclose(loss, want, rtol=5e-5, atol=1e-7)
    g = _grads(m, eng)
    for k in gw:
        assert rel_l2(g[k], gw[k]) < 2e-4, (k, rel_l2(g[k], gw[k]))


def test_wide_cfg5_bf16_matches_bf16_emulation(cvae):
    """bf16 kernels at the cfg5 shape against the CPU emulation of their rounding points (tight),
    and against the fp32 reference (the bf16 operand-rounding distance, loose)."""
    B = 64
    ref, m, eng, x, eps = _wide(cvae, "bf16", B)
    x = x.to(torch.bfloat16).float()
    loss = eng.forward_backward(x, eps=eps).cpu().numpy()
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    ne, nd = WIDE["n_enc"], WIDE["n_dec"]
    r, mu, lv, hc, c = cvae_np.forward(p, x.numpy(), eps.numpy(), n_enc=ne, n_dec=nd, q=cvae_np.bf16)
    np.testing.assert_allclose(loss, cvae_np.losses(r, c["rel"], mu, lv), rtol=3e-3, atol=1e-6)
    gw = cvae_np.backward(p, c, r, mu, lv, n_enc=ne, n_dec=nd)
    g = _grads(m, eng)
    for k in cvae_np.param_keys(ne, nd):
        assert rel_l2(g[k], gw[k]) < 3e-2, (k, rel_l2(g[k], gw[k]))
    want, _ = _oracle_grads(ref, x, eps)
    np.testing.assert_allclose(loss, want, rtol=3e-2, atol=1e-6)


def test_wide_cfg5_bf16_training_full_batch(cvae):
    """B=1024 at the cfg5 shape: the fused train step stays finite and lowers the ELBO; the
    two-launch split path (data-parallel route) equals it bit for bit."""
    ref, m, eng, x, _ = _wide(cvae, "bf16", 1024)
    m2 = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    m2.load_state_dict(ref.state_dict())
    e2 = m2.attach(dtype="bf16", max_batch=1024, device="cuda:0")
    x = x.cuda()
    eps = torch.randn(1024, WIDE["Z"], generator=torch.Generator().manual_seed(7))
    for _ in range(3):
        eng.train_step(x, eps=eps)
        e2.forward_backward(x, eps=eps)
        e2.adam_step(1.0)
    torch.cuda.synchronize()
    assert torch.equal(eng.params, e2.params)
    first = eng.train_step(x).clone()
    for _ in range(30):
        last = eng.train_step(x)
    torch.cuda.synchronize()
    assert torch.isfinite(eng.params).all()
    assert float(last[0]) < float(first[0])


def test_wide_cfg5_generate(cvae):
    """Batched generation (decode mode) at the cfg5 shape vs the oracle decoder."""
    ref, m, eng, _, _ = _wide(cvae, "fp32", 48)
    st = torch.randn(48, 2) * 20
    z = torch.randn(48, WIDE["Z"])
    rel, ab = m.generate(st, z=z.cuda())
    with torch.no_grad():
        want = ref.decode(z, ref.condition_encoder(st))
    assert rel_l2(rel.cpu().numpy(), want.numpy()) < 1e-5


def _wide_pair(cvae, monkeypatch, B, seed=0):
    """Two bf16 engines at the cfg5 shape on the same weights: the specialised wide chain
    (cvae_widechain.h) and the generic interpreter (CVAE_GENERIC=1 at creation)."""
    ref, m, eng, x, eps = _wide(cvae, "bf16", B, seed)
    monkeypatch.setenv("CVAE_GENERIC", "1")
    m2 = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    m2.load_state_dict(ref.state_dict())
    e2 = m2.attach(dtype="bf16", max_batch=max(B, 32), device="cuda:0")
    monkeypatch.delenv("CVAE_GENERIC")
    assert eng.train_kernel == "wide" and e2.train_kernel == "generic"
    return ref, m, eng, m2, e2, x, eps


@pytest.mark.parametrize("B", [37, 200])
def test_wide_chain_matches_generic_and_emulation(cvae, monkeypatch, B):
    """The specialised cfg5 row chain against the generic interpreter (same rounding points, fp32
    summation order aside) and against the CPU emulation of those rounding points, ragged last
    tile (B=37) and a gathered batch (B=200 rows of 300 by index)."""
    ref, m, eng, m2, e2, x, eps = _wide_pair(cvae, monkeypatch, B)
    x = x.to(torch.bfloat16).float()
    if B == 200:
        pool = torch.randn(300, WIDE["S"], WIDE["D"], generator=torch.Generator().manual_seed(9)).to(torch.bfloat16)
        idx = torch.randperm(300, generator=torch.Generator().manual_seed(3))[:B]
        x = pool[idx].float()
        lw = eng.forward_backward(pool.cuda(), idx=idx.cuda(), eps=eps).cpu().numpy()
    else:
        lw = eng.forward_backward(x, eps=eps).cpu().numpy()
    lg = e2.forward_backward(x, eps=eps).cpu().numpy()
    np.testing.assert_allclose(lw, lg, rtol=2e-3, atol=1e-6)
    gw, gg = _grads(m, eng), _grads(m2, e2)
    for k in gw:
        assert rel_l2(gw[k], gg[k]) < 1e-2, (k, rel_l2(gw[k], gg[k]))
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    ne, nd = WIDE["n_enc"], WIDE["n_dec"]
    r, mu, lv, hc, c = cvae_np.forward(p, x.numpy(), eps.numpy(), n_enc=ne, n_dec=nd, q=cvae_np.bf16)
    np.testing.assert_allclose(lw, cvae_np.losses(r, c["rel"], mu, lv), rtol=3e-3, atol=1e-6)
    ge = cvae_np.backward(p, c, r, mu, lv, n_enc=ne, n_dec=nd)
    for k in cvae_np.param_keys(ne, nd):
        assert rel_l2(gw[k], ge[k]) < 3e-2, (k, rel_l2(gw[k], ge[k]))


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
@pytest.mark.parametrize("B", [64, 1000])
def test_wide_chain_repeatable_and_dw_tiles_bit_equal(cvae, monkeypatch, dtype, B):
    """The wide chain is race-free: eight forward_backward calls on the same input give bit-equal
    gradients and losses (an inline-asm store hazard once corrupted whole gradient columns in
    14-22 of 40 calls).  The dW launch's 32 x 64 tiles (the default for this long tile list:
    widewgrad_kernel), the generic kernel over them (CVAE_GENERIC_DW=1) and 32 x 32 tiles
    (CVAE_DW_NI2=0) give the same bits: each element is the same K sum in the same chunk order and
    the same fixed-order cross-wave sum.  B = 1000: a ragged last row tile."""
    ref, m, eng, x, eps = _wide(cvae, dtype, B)
    monkeypatch.setenv("CVAE_DW_NI2", "0")
    m2 = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    m2.load_state_dict(ref.state_dict())
    e2 = m2.attach(dtype=dtype, max_batch=B, device="cuda:0")
    monkeypatch.delenv("CVAE_DW_NI2")
    xd = x.to("cuda", torch.bfloat16)
    l0 = eng.forward_backward(xd, eps=eps).clone()
    g0 = eng.grads.clone()
    for _ in range(7):
        l = eng.forward_backward(xd, eps=eps)
        assert torch.equal(l, l0) and torch.equal(eng.grads, g0)
    e2.forward_backward(xd, eps=eps)
    assert torch.equal(e2.grads, g0)
    # a fused training step (dW ⊕ Adam) on fresh engines (forward_backward advances the step count):
    # the compile-time tile decode of the wide shape (widewgrad_kernel, the default), the generic
    # kernel over the same 32 x 64 tile list (CVAE_GENERIC_DW=1) and 32 x 32 tiles (CVAE_DW_NI2=0)
    fresh = []
    for env in (None, ("CVAE_DW_NI2", "0"), ("CVAE_GENERIC_DW", "1")):
        if env:
            monkeypatch.setenv(*env)
        mm = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
        mm.load_state_dict(ref.state_dict())
        ee = mm.attach(dtype=dtype, max_batch=B, device="cuda:0")
        if env:
            monkeypatch.delenv(env[0])
        for _ in range(2):
            ee.train_step(xd, eps=eps)
        fresh.append(ee)
    torch.cuda.synchronize()
    a3 = fresh[0]
    for a4 in fresh[1:]:
        assert torch.equal(a3.params, a4.params) and torch.equal(a3.m, a4.m) and torch.equal(a3.v, a4.v)
        assert torch.equal(a3.loss, a4.loss) and torch.equal(a3.counters, a4.counters)


def test_wide_fp8_chain_repeatable_stress(cvae):
    """200 forward_backward calls of the e4m3 wide chain on one input give the same bits.  Its
    weight fragments are buffer loads with a 16-state pad after every e4m3 MFMA (f8_pad,
    cvae_widechain.h): without the pad every call differed (the refill load wrote ring registers a
    queued e4m3 MFMA had not read yet; scripts/repeat_check.py, profiles/r05i/)."""
    ref, m, eng, x, eps = _wide(cvae, "fp8", 64)
    xd = x.to("cuda", torch.bfloat16)
    l0 = eng.forward_backward(xd, eps=eps).clone()
    g0 = eng.grads.clone()
    bad = 0
    for _ in range(200):
        l = eng.forward_backward(xd, eps=eps)
        bad += 0 if torch.equal(l, l0) and torch.equal(eng.grads, g0) else 1
    torch.cuda.synchronize()
    assert bad == 0, f"{bad} of 200 calls differ"


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_wide_dw_decode_split_k_equals_generic(cvae, monkeypatch, dtype):
    """B = 8192 at the cfg5 shape: the dW launch splits K (the batch) over 4 blocks per tile with the
    sc1 ticket hand-off; the compile-time tile decode (widewgrad_kernel) and the generic tile-list
    kernel (CVAE_GENERIC_DW=1) give the same bits over two training steps (params, moments,
    loss, counters)."""
    B = 8192
    torch.manual_seed(0)
    ref = OracleCVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    engines = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("CVAE_GENERIC_DW", env)
        mm = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
        mm.load_state_dict(ref.state_dict())
        engines.append(mm.attach(dtype=dtype, max_batch=B, device="cuda:0"))
        monkeypatch.delenv("CVAE_GENERIC_DW", raising=False)
    xd = torch.randn(B, WIDE["S"], WIDE["D"], generator=torch.Generator().manual_seed(11)).to("cuda", torch.bfloat16)
    for _ in range(2):
        for e in engines:
            e.train_step(xd)
    torch.cuda.synchronize()
    a, b = engines
    assert torch.isfinite(a.loss).all()
    assert torch.equal(a.params, b.params) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
    assert torch.equal(a.loss, b.loss) and torch.equal(a.counters, b.counters)


def test_wide_chain_philox_and_training_match_generic(cvae, monkeypatch):
    """In-kernel Philox eps (keyed by the global row: eps_row0) draws the same noise in the wide
    chain as in the generic interpreter; three full training steps (dW ⊕ Adam behind each chain)
    stay within the bf16 summation-order distance of the generic run; and the wide chain is
    deterministic (two identical runs are bit-equal)."""
    B = 96
    ref, m, eng, m2, e2, x, _ = _wide_pair(cvae, monkeypatch, B)
    xd = x.to("cuda", torch.bfloat16)
    lw = eng.forward_backward(xd, row0=640).cpu().numpy()
    lg = e2.forward_backward(xd, row0=640).cpu().numpy()
    np.testing.assert_allclose(lw, lg, rtol=2e-3, atol=1e-6)
    gw, gg = _grads(m, eng), _grads(m2, e2)
    for k in gw:
        assert rel_l2(gw[k], gg[k]) < 1e-2, (k, rel_l2(gw[k], gg[k]))
    p0 = eng.params.clone()
    for _ in range(3):
        eng.train_step(xd)
        e2.train_step(xd)
    torch.cuda.synchronize()
    np.testing.assert_allclose(eng.loss.cpu().numpy(), e2.loss.cpu().numpy(), rtol=3e-3, atol=1e-6)
    dp = (eng.params - e2.params).norm() / (eng.params - p0).norm()
    assert float(dp) < 2e-2, float(dp)
    # determinism: a second wide engine from the same state replays bit for bit
    m3 = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    m3.load_state_dict(ref.state_dict())
    e3 = m3.attach(dtype="bf16", max_batch=B, device="cuda:0")
    e3.forward_backward(xd, row0=640)
    for _ in range(3):
        e3.train_step(xd)
    torch.cuda.synchronize()
    assert torch.equal(e3.params, eng.params) and torch.equal(e3.loss, eng.loss)


def test_train_cli_end_to_end(cvae, golden, tmp_path):
    """python -m cvae_amd.train (the reference __main__ as a CLI): two epochs on the sce1 rows,
    checkpoint with the 24 reference keys and the loss CSV written."""
    from cvae_amd.train import main
    data = tmp_path / "trajectory_sce1_cond.npy"
    np.save(data, golden("sce_fixed.npz")["sce1_x"].astype(np.float64))
    mo, lo = tmp_path / "m.pth", tmp_path / "loss.png"
    main(["--data", str(data), "--epochs", "2", "--seed", "0", "--model-out", str(mo), "--loss-out", str(lo)])
    sd = torch.load(mo, weights_only=True)
    assert list(sd.keys()) == list(OracleCVAE(10, 3, 8).state_dict().keys())
    rows = (tmp_path / "loss.csv").read_text().strip().splitlines()
    assert rows[0].split(",")[0] == "total_loss" and len(rows) == 3


def test_bf16_200_step_loss_curve_vs_fp32_oracle(cvae):
    """the bf16 path's 200-step training curve at the cfg2 shape stays within 2 % of
    the fp32 reference trained on the same batches and the same eps (B=256, one fixed batch
    per step drawn from a 2048-row synthetic set)."""
    from oracle.cvae_oracle import oracle_step
    torch.manual_seed(0)
    ref = OracleCVAE(100, 6, 8)
    m, eng = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=256)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    gen = torch.Generator().manual_seed(1234)
    data = torch.randn(2048, 100, 6, generator=gen).to(torch.bfloat16).float()
    data_dev = data.cuda()
    got, want = [], []
    for t in range(200):
        idx = torch.randint(0, 2048, (256,), generator=gen)
        eps = torch.randn(256, 8, generator=gen)
        got.append(eng.train_step(data_dev, idx=idx.cuda(), eps=eps).cpu().numpy().copy())
        want.append(oracle_step(ref, opt, data[idx], weights=W, eps=eps))
    got, want = np.array(got), np.array(want)
    assert want[-1, 0] < 0.8 * want[0, 0]  # the reference run itself trains (0.169 → 0.116)
    # the curve (10-step means) within 2 %; single steps within 3 % (measured max 2.2 %, step ~190)
    sm = lambda a: a.reshape(20, 10).mean(1)  # noqa: E731
    np.testing.assert_allclose(sm(got[:, 0]), sm(want[:, 0]), rtol=2e-2)
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=3e-2)


# ---- fp8 forward GEMMs (CVAE_FP8, BASELINE cfg5 "fp8 MFMA GEMMs").  Layers whose padded K is a
# multiple of 64 multiply e4m3(bf16 X) by e4m3(s·W) (v_mfma_f32_16x16x32_fp8_fp8); the rest of
# the step is the bf16 path.  Checked against the CPU emulation of exactly those rounding points;
# the distance to the fp32 reference is printed (a measured deviation, not a parity claim).
FP8_SHAPES = {"cfg2": dict(S=100, D=6, Z=8, n_enc=4, n_dec=4), "cfg5": WIDE}

# Gradient rel-L2 bounds of the fp8 paths against the CPU emulation of their rounding points,
# (max over tensors, median over tensors, max over every tensor but decoder.0.weight): about 2x the
# maxima measured on the MI355X (rounds 4-5, profiles/r04y, profiles/r05b; printed by every run).
# An emulation of e4m3 rounding points is not bit-exact — the kernels accumulate in another order,
# and an element whose pre-rounding value lands on the other side of a rounding boundary moves by
# one e4m3 ulp (6 %) — so these bounds sit above bf16's 3e-2 where the flips compound:
#   cfg2 (generic fp8 interpreter, bf16 backward): max 0.009, median 0.0022;
#   cfg5 wide chain: max 0.0424-0.0640 — decoder.0.weight every time, with the MX dX GEMMs and with
#   bf16 ones alike (so the e4m3 forward's flips, not the MX backward: its input [z ‖ h_c] and its
#   gradient sit at the end of the 16 e4m3 forward layers and the reparameterisation) — every other
#   tensor <= 0.0275, median 0.0019-0.0041.
FP8_EMU_BOUNDS = {"cfg2": (2e-2, 5e-3, 2e-2), "cfg5": (1.3e-1, 1e-2, 5.5e-2)}


def _fp8_bounds(errs, what, bounds):
    mx, med, rest = bounds
    vals = list(errs.values())
    others = [v for k, v in errs.items() if k != "decoder.0.weight"]
    print(f"{what}: max {max(vals):.4f} ({max(errs, key=errs.get)}), median {np.median(vals):.4f}, "
          f"max without decoder.0.weight {max(others):.4f}")
    assert max(vals) < mx and np.median(vals) < med and max(others) < rest, errs


@pytest.mark.parametrize("shape", ["cfg2", "cfg5"])
def test_fp8_matches_fp8_emulation(cvae, shape):
    c = FP8_SHAPES[shape]
    B = 64
    torch.manual_seed(0)
    ref = OracleCVAE(c["S"], c["D"], c["Z"], 128, c["n_enc"], c["n_dec"])
    m = cvae.ConditionalTrajectoryVAE(c["S"], c["D"], c["Z"], 128, c["n_enc"], c["n_dec"])
    m.load_state_dict(ref.state_dict())
    eng = m.attach(dtype="fp8", max_batch=B, device="cuda:0")
    x = torch.randn(B, c["S"], c["D"], generator=torch.Generator().manual_seed(1234)).to(torch.bfloat16).float()
    eps = torch.randn(B, c["Z"], generator=torch.Generator().manual_seed(4321))
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    ne, nd = c["n_enc"], c["n_dec"]
    f8 = cvae_np.fp8_layers(p, c["S"], c["D"], c["Z"], 128, ne, nd)
    assert "fc_mu" in f8 and "encoder.3" in f8  # the K=128/256 layers run in fp8 at both shapes
    r, mu, lv, hc, cc = cvae_np.forward(p, x.numpy(), eps.numpy(), n_enc=ne, n_dec=nd, q=cvae_np.bf16, f8=f8)
    out = eng.forward(x, eps=eps)
    got_r = out[0].cpu().numpy()
    assert rel_l2(got_r, r) < 1e-2, rel_l2(got_r, r)
    loss = eng.forward_backward(x, eps=eps).cpu().numpy()
    want = cvae_np.losses(r, cc["rel"], mu, lv)
    np.testing.assert_allclose(loss, want, rtol=5e-3, atol=1e-6)
    # the cfg5 shape runs the wide chain: its large dX GEMMs are e4m3 with MX row-block scales
    f8b = cvae_np.fp8b_layers(p, c["S"], c["D"], c["Z"], 128, ne, nd) if eng.train_kernel == "wide" else None
    assert (shape == "cfg5") == bool(f8b)
    gw = cvae_np.backward(p, cc, r, mu, lv, n_enc=ne, n_dec=nd, f8b=f8b)
    g = _grads(m, eng)
    errs = {k: rel_l2(g[k], gw[k]) for k in cvae_np.param_keys(ne, nd)}
    print(f"fp8 {shape}: grad rel-L2 vs emulation", {k: round(v, 4) for k, v in errs.items()})
    _fp8_bounds(errs, f"fp8 {shape} vs emulation", FP8_EMU_BOUNDS[shape])
    want32, _ = _oracle_grads(ref, x, eps)
    dev = np.abs(loss - want32) / np.abs(want32)
    print(f"fp8 {shape}: loss rel deviation from the fp32 reference {dev}")
    assert (dev < 0.25).all(), dev


@pytest.mark.parametrize("B", [37, 200])
def test_wide_fp8_chain_matches_generic_fp8(cvae, monkeypatch, B):
    """The cfg5 fp8 form of the wide chain (e4m3 activation twins written by the producing
    epilogues, e4m3 weight pairs in the ring; the dX GEMMs of the last decoder layer, decoder L0 and
    fc in e4m3 with MX row-block scales) against the generic interpreter's fp8 path (CVAE_GENERIC=1:
    the same forward rounding points, a bf16 backward) — losses tight, gradients within the e4m3
    backward's rounding (printed) — and against the CPU emulation of exactly its rounding points
    (cvae_np fp8 forward + mx_dx; emulation tolerances of test_fp8_matches_fp8_emulation); ragged
    tile (B=37) and a gathered batch (B=200)."""
    ref, m, eng, x, eps = _wide(cvae, "fp8", B)
    monkeypatch.setenv("CVAE_GENERIC", "1")
    m2 = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    m2.load_state_dict(ref.state_dict())
    e2 = m2.attach(dtype="fp8", max_batch=max(B, 32), device="cuda:0")
    monkeypatch.delenv("CVAE_GENERIC")
    assert eng.train_kernel == "wide" and e2.train_kernel == "generic"
    x = x.to(torch.bfloat16).float()
    if B == 200:
        pool = torch.randn(300, WIDE["S"], WIDE["D"], generator=torch.Generator().manual_seed(9)).to(torch.bfloat16)
        idx = torch.randperm(300, generator=torch.Generator().manual_seed(3))[:B]
        x = pool[idx].float()
        lw = eng.forward_backward(pool.cuda(), idx=idx.cuda(), eps=eps).cpu().numpy()
    else:
        lw = eng.forward_backward(x, eps=eps).cpu().numpy()
    lg = e2.forward_backward(x, eps=eps).cpu().numpy()
    np.testing.assert_allclose(lw, lg, rtol=5e-3, atol=1e-6)
    gw, gg = _grads(m, eng), _grads(m2, e2)
    errs = {k: rel_l2(gw[k], gg[k]) for k in gw}
    print(f"wide fp8 chain B={B}: grad rel-L2 vs the generic bf16 backward", {k: round(v, 4) for k, v in errs.items()})
    # the MX dX GEMMs against a bf16 backward: measured max 0.0424-0.0466 (decoder.0.bias), median 0.020
    print(f"  max {max(errs.values()):.4f}, median {np.median(list(errs.values())):.4f}")
    assert max(errs.values()) < 0.1 and np.median(list(errs.values())) < 0.04, errs
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    ne, nd = WIDE["n_enc"], WIDE["n_dec"]
    f8 = cvae_np.fp8_layers(p, WIDE["S"], WIDE["D"], WIDE["Z"], 128, ne, nd)
    f8b = cvae_np.fp8b_layers(p, WIDE["S"], WIDE["D"], WIDE["Z"], 128, ne, nd)
    assert sorted(f8b) == ["decoder.0", f"decoder.{2 * (nd - 1)}", "fc_logvar", "fc_mu"], sorted(f8b)
    r, mu, lv, hc, cc = cvae_np.forward(p, x.numpy(), eps.numpy(), n_enc=ne, n_dec=nd, q=cvae_np.bf16, f8=f8)
    np.testing.assert_allclose(lw, cvae_np.losses(r, cc["rel"], mu, lv), rtol=5e-3, atol=1e-6)
    ge = cvae_np.backward(p, cc, r, mu, lv, n_enc=ne, n_dec=nd, f8b=f8b)
    errs = {k: rel_l2(gw[k], ge[k]) for k in cvae_np.param_keys(ne, nd)}
    print(f"wide fp8 chain B={B}: grad rel-L2 vs emulation", {k: round(v, 4) for k, v in errs.items()})
    _fp8_bounds(errs, f"wide fp8 chain B={B} vs emulation", FP8_EMU_BOUNDS["cfg5"])
    gb = cvae_np.backward(p, cc, r, mu, lv, n_enc=ne, n_dec=nd)  # the same forward, a bf16 backward
    dev = {k: rel_l2(ge[k], gb[k]) for k in cvae_np.param_keys(ne, nd)}
    print(f"  emulation: MX e4m3 dX vs bf16 dX, grad rel-L2 median {np.median(list(dev.values())):.4f} "
          f"max {max(dev.values()):.4f}")
    # what the MX dX GEMMs cost in accuracy, on the CPU: measured median 0.0196-0.0199,
    # max 0.0423-0.0470 (profiles/r04y)
    assert max(dev.values()) < 0.1 and np.median(list(dev.values())) < 0.04, dev


@pytest.mark.parametrize("B", [37, 200])
def test_wide_fp8_bf16_dx_fallback(cvae, monkeypatch, B):
    """CVAE_FP8_DX=bf16 at creation: the wide chain keeps its e4m3 forward GEMMs and
    runs every dX GEMM in bf16 (wchain::Cfg5F8B, no e4m3 Wᵀ copies) — the rounding points of the
    generic interpreter's fp8 path.  Against it: losses rtol 1e-4, gradients rel-L2 < 1e-3 (the
    same rounding points; measured < 5e-5); against the CPU emulation without MX dX, the bounds of
    the fp8 emulation tests."""
    monkeypatch.setenv("CVAE_FP8_DX", "bf16")
    ref, m, eng, x, eps = _wide(cvae, "fp8", B)
    monkeypatch.setenv("CVAE_GENERIC", "1")
    m2 = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    m2.load_state_dict(ref.state_dict())
    e2 = m2.attach(dtype="fp8", max_batch=max(B, 32), device="cuda:0")
    monkeypatch.delenv("CVAE_GENERIC")
    monkeypatch.delenv("CVAE_FP8_DX")
    assert eng.train_kernel == "wide" and e2.train_kernel == "generic"
    x = x.to(torch.bfloat16).float()
    lw = eng.forward_backward(x, eps=eps).cpu().numpy()
    lg = e2.forward_backward(x, eps=eps).cpu().numpy()
    np.testing.assert_allclose(lw, lg, rtol=1e-4, atol=1e-7)
    gw, gg = _grads(m, eng), _grads(m2, e2)
    errs = {k: rel_l2(gw[k], gg[k]) for k in gw}
    print(f"wide fp8 chain, bf16 dX, B={B}: grad rel-L2 vs the generic fp8 path: max {max(errs.values()):.2e} "
          f"({max(errs, key=errs.get)}), median {np.median(list(errs.values())):.2e}")
    # the same rounding points in another accumulation order: measured max < 5e-5 (profiles/r05b)
    assert max(errs.values()) < 1e-3, errs
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    ne, nd = WIDE["n_enc"], WIDE["n_dec"]
    f8 = cvae_np.fp8_layers(p, WIDE["S"], WIDE["D"], WIDE["Z"], 128, ne, nd)
    r, mu, lv, hc, cc = cvae_np.forward(p, x.numpy(), eps.numpy(), n_enc=ne, n_dec=nd, q=cvae_np.bf16, f8=f8)
    ge = cvae_np.backward(p, cc, r, mu, lv, n_enc=ne, n_dec=nd)
    errs = {k: rel_l2(gw[k], ge[k]) for k in cvae_np.param_keys(ne, nd)}
    _fp8_bounds(errs, f"wide fp8 chain, bf16 dX, B={B} vs emulation", FP8_EMU_BOUNDS["cfg5"])


def test_fp8_mx_dx_loss_trajectory_vs_bf16_dx(cvae, monkeypatch):
    """What the MX e4m3 dX GEMMs cost a training run: 40 steps of the cfg5 fp8 step
    (B=256, Philox eps, one seeded batch pool) with MX dX against the same run with bf16 dX
    (CVAE_FP8_DX=bf16), same init and batches: the loss curves (10-step means of the total ELBO)
    within 2 %, every step within 5 %; both runs train.  Deviations printed."""
    B, pool = 256, 1024
    xs = torch.randn(pool, WIDE["S"], WIDE["D"], generator=torch.Generator().manual_seed(5)).cuda()
    gen = torch.Generator().manual_seed(6)
    idxs = [torch.randint(0, pool, (B,), generator=gen).cuda() for _ in range(40)]
    curves = {}
    for form in ("mx", "bf16"):
        if form == "bf16":
            monkeypatch.setenv("CVAE_FP8_DX", "bf16")
        ref, m, eng, _, _ = _wide(cvae, "fp8", B)
        monkeypatch.delenv("CVAE_FP8_DX", raising=False)
        xin = eng.as_input(xs)
        curves[form] = np.array([eng.train_step(xin, idx=i).cpu().numpy()[0] for i in idxs])
    a, b = curves["mx"], curves["bf16"]
    sm = lambda v: v.reshape(4, 10).mean(1)  # noqa: E731
    print(f"cfg5 fp8 40 steps: MX dX {a[0]:.5f} -> {a[-1]:.5f}, bf16 dX {b[0]:.5f} -> {b[-1]:.5f}; "
          f"max step rel dev {np.max(np.abs(a - b) / np.abs(b)):.4f}, "
          f"10-step means rel dev {np.max(np.abs(sm(a) - sm(b)) / np.abs(sm(b))):.4f}")
    assert np.isfinite(a).all() and a[-10:].mean() < a[:10].mean() and b[-10:].mean() < b[:10].mean()
    np.testing.assert_allclose(sm(a), sm(b), rtol=2e-2)
    np.testing.assert_allclose(a, b, rtol=5e-2)


@pytest.mark.parametrize("B", [256, 1024])
def test_wide_fp8_mx_dw_matches_emulation(cvae, monkeypatch, B):
    """CVAE_FP8_DW=mx (BASELINE configs[4] "fp8 MFMA GEMMs" for the weight gradients,
    Training_VAE.py:141-167 via :362): every 32 × 64 dW tile multiplies e4m3 operands with MX
    scales over 32-row blocks of the batch (cvae_wgrad.h mx_dw_chunk).  Against the CPU emulation
    of those rounding points (oracle mx_dw on the emulated bf16 arena rows): the fp8 emulation
    bounds; the same gradients sit closer to it than to the bf16-dW emulation (the MX path ran).
    The fused step equals the split (data-parallel) step bit for bit."""
    monkeypatch.setenv("CVAE_FP8_DW", "mx")
    ref, m, eng, x, eps = _wide(cvae, "fp8", B)
    ef, es = [], []
    for lst in (ef, es):  # fresh engines (device step counters at 0) for the fused / split comparison
        mm = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
        mm.load_state_dict(ref.state_dict())
        lst.append(mm.attach(dtype="fp8", max_batch=B, device="cuda:0"))
    e1, e2 = ef[0], es[0]
    monkeypatch.delenv("CVAE_FP8_DW")
    assert eng.train_kernel == "wide"
    x = x.to(torch.bfloat16).float()
    lw = eng.forward_backward(x, eps=eps).cpu().numpy()
    gw = _grads(m, eng)
    p = {k: v.numpy() for k, v in ref.state_dict().items()}
    ne, nd = WIDE["n_enc"], WIDE["n_dec"]
    f8 = cvae_np.fp8_layers(p, WIDE["S"], WIDE["D"], WIDE["Z"], 128, ne, nd)
    f8b = cvae_np.fp8b_layers(p, WIDE["S"], WIDE["D"], WIDE["Z"], 128, ne, nd)
    mxw = cvae_np.mxw_layers(p, ne, nd)
    r, mu, lv, hc, cc = cvae_np.forward(p, x.numpy(), eps.numpy(), n_enc=ne, n_dec=nd, q=cvae_np.bf16, f8=f8)
    np.testing.assert_allclose(lw, cvae_np.losses(r, cc["rel"], mu, lv), rtol=5e-3, atol=1e-6)
    gx = cvae_np.backward(p, cc, r, mu, lv, n_enc=ne, n_dec=nd, f8b=f8b, mxw=mxw)
    gb = cvae_np.backward(p, cc, r, mu, lv, n_enc=ne, n_dec=nd, f8b=f8b)
    errs = {k: rel_l2(gw[k], gx[k]) for k in cvae_np.param_keys(ne, nd)}
    _fp8_bounds(errs, f"wide fp8 MX dW B={B} vs emulation", FP8_EMU_BOUNDS["cfg5"])
    wk = [n + ".weight" for n in sorted(mxw)]
    e_mx = np.median([rel_l2(gw[k], gx[k]) for k in wk])
    e_bf = np.median([rel_l2(gw[k], gb[k]) for k in wk])
    dev = {k: rel_l2(gx[k], gb[k]) for k in wk}
    print(f"  MX-dW weights: median rel-L2 vs MX emulation {e_mx:.4f}, vs bf16-dW emulation {e_bf:.4f}; "
          f"emulation MX dW vs bf16 dW median {np.median(list(dev.values())):.4f} max {max(dev.values()):.4f}")
    assert e_mx < e_bf
    assert max(dev.values()) < 0.1 and np.median(list(dev.values())) < 0.05, dev
    for _ in range(2):  # fused step == split step, MX dW in both (PM_ADAM and PM_GRAD forms)
        e1.train_step(x, eps=eps)
        e2.forward_backward(x, eps=eps)
        e2.adam_step(1.0)
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params)


def test_fp8_mx_dw_loss_trajectory_vs_bf16_dw(cvae, monkeypatch):
    """The MX dW over a training run: 40 cfg5 fp8 steps (B=256) with CVAE_FP8_DW=mx against the
    default bf16 dW, same init and batches: 10-step means of the ELBO within 2 %, every step within
    5 %, both runs train (deviations printed)."""
    B, pool = 256, 1024
    xs = torch.randn(pool, WIDE["S"], WIDE["D"], generator=torch.Generator().manual_seed(5)).cuda()
    gen = torch.Generator().manual_seed(6)
    idxs = [torch.randint(0, pool, (B,), generator=gen).cuda() for _ in range(40)]
    curves = {}
    for form in ("mx", "bf16"):
        if form == "mx":
            monkeypatch.setenv("CVAE_FP8_DW", "mx")
        ref, m, eng, _, _ = _wide(cvae, "fp8", B)
        monkeypatch.delenv("CVAE_FP8_DW", raising=False)
        xin = eng.as_input(xs)
        curves[form] = np.array([eng.train_step(xin, idx=i).cpu().numpy()[0] for i in idxs])
    a, b = curves["mx"], curves["bf16"]
    sm = lambda v: v.reshape(4, 10).mean(1)  # noqa: E731
    print(f"cfg5 fp8 40 steps: MX dW {a[0]:.5f} -> {a[-1]:.5f}, bf16 dW {b[0]:.5f} -> {b[-1]:.5f}; "
          f"max step rel dev {np.max(np.abs(a - b) / np.abs(b)):.4f}, "
          f"10-step means rel dev {np.max(np.abs(sm(a) - sm(b)) / np.abs(sm(b))):.4f}")
    assert np.isfinite(a).all() and a[-10:].mean() < a[:10].mean() and b[-10:].mean() < b[:10].mean()
    np.testing.assert_allclose(sm(a), sm(b), rtol=2e-2)
    np.testing.assert_allclose(a, b, rtol=5e-2)


def test_fp8_training_full_batch_cfg5(cvae):
    """B=1024 at the cfg5 shape in fp8: the fused step (Adam writes e4m3 operand copies with the
    packed scales) equals the two-launch split path bit for bit, stays finite and lowers the ELBO."""
    ref, m, eng, x, _ = _wide(cvae, "fp8", 1024)
    m2 = cvae.ConditionalTrajectoryVAE(WIDE["S"], WIDE["D"], WIDE["Z"], 128, WIDE["n_enc"], WIDE["n_dec"])
    m2.load_state_dict(ref.state_dict())
    e2 = m2.attach(dtype="fp8", max_batch=1024, device="cuda:0")
    x = x.cuda()
    eps = torch.randn(1024, WIDE["Z"], generator=torch.Generator().manual_seed(7))
    for _ in range(3):
        eng.train_step(x, eps=eps)
        e2.forward_backward(x, eps=eps)
        e2.adam_step(1.0)
    torch.cuda.synchronize()
    assert torch.equal(eng.params, e2.params)
    first = eng.train_step(x).clone()
    for _ in range(30):
        last = eng.train_step(x)
    torch.cuda.synchronize()
    assert torch.isfinite(eng.params).all()
    assert float(last[0]) < float(first[0])



def test_rccl_allreduce_split_step_equals_fused(cvae):
    """The DP step's exchange on the real backend: fwd/bwd → RCCL all_reduce (the "nccl" backend,
    a world-1 group on this one-GPU box) → Adam, plus the epoch loss all_reduce, equals the fused
    step bit for bit (cvae_amd/dist.py DataParallelStep; Training_VAE.py:351-363)."""
    import os
    import torch.distributed as tdist
    from cvae_amd import dist as dp
    from conftest import free_port
    assert not tdist.is_initialized()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0,
                             world_size=1, device_id=torch.device("cuda", 0))
    try:
        torch.manual_seed(0)
        ref = OracleCVAE(100, 6, 8)
        m1, e1 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=256)
        m2, e2 = _model(cvae, 100, 6, 8, sd=ref.state_dict(), dtype="bf16", max_batch=256)
        step = dp.DataParallelStep(e2)
        step.broadcast_params()
        x = e1.as_input(torch.randn(256, 100, 6, generator=torch.Generator().manual_seed(7)))
        eps = torch.randn(256, 8, generator=torch.Generator().manual_seed(8)).cuda()
        for _ in range(3):
            e1.train_step(x, eps=eps)
            e2.forward_backward(x, eps=eps)
            tdist.all_reduce(e2.grads, op=tdist.ReduceOp.SUM)
            e2.adam_step(1.0)
        acc1 = e1.loss_accum.clone()
        acc2 = step.epoch_loss_sums()
        torch.cuda.synchronize()
        assert torch.equal(e1.params, e2.params)
        assert torch.equal(e1.m, e2.m) and torch.equal(e1.v, e2.v)
        assert torch.equal(acc1, acc2) and float(e2.loss_accum.abs().sum()) == 0.0
    finally:
        tdist.destroy_process_group()



@pytest.mark.parametrize("B", [1024, 8192])
def test_dw_buckets_equal_whole_launch(cvae, monkeypatch, B):
    """The two dW buckets of the RCCL data-parallel step (fchain::fastwgrad_bucket_kernel: the
    decoder tail of the tile list with the chain, then the rest) give the whole dW launch's gradient
    bit for bit — also with split-K (B = 8192) — and so do the generic tile-list buckets
    (CVAE_GENERIC_BUCKETS=1).  Host eps: every call draws the same noise."""
    torch.manual_seed(0)
    ref = cvae.ConditionalTrajectoryVAE(100, 6, 8)
    engines = []
    for v in ("0", "1"):
        monkeypatch.setenv("CVAE_GENERIC_BUCKETS", v)
        m = cvae.ConditionalTrajectoryVAE(100, 6, 8)
        m.load_state_dict(ref.state_dict())
        engines.append(m.attach(dtype="bf16", max_batch=B, device="cuda:0"))
    monkeypatch.delenv("CVAE_GENERIC_BUCKETS")
    x = engines[0].as_input(torch.randn(B, 100, 6, generator=torch.Generator().manual_seed(5)))
    eps = torch.randn(B, 8, generator=torch.Generator().manual_seed(6)).cuda()
    e = engines[0]
    e.forward_backward(x, eps=eps)  # CVAE_PART_ALL: one dW launch
    torch.cuda.synchronize()
    g_all, l_all = e.grads.clone(), e.loss.clone()
    for eng in engines:
        eng.grads.fill_(float("nan"))
        eng.forward_backward(x, eps=eps, parts=3)  # chain + decoder bucket
        eng.wgrad_rest(B)
        torch.cuda.synchronize()
        assert torch.equal(eng.grads, g_all)
        assert torch.equal(eng.loss, l_all)


def test_kernel_dispatch_per_configuration(cvae):
    """Which row chain and which dW ⊕ Adam kernel each BASELINE configuration's handle runs
    (cvae_train_kernel / cvae_dw_kernel): the specialised kernels, never the generic interpreter;
    and the chain's rows per workgroup (cvae_chain_rows): 4 for the fp32 chain up to 1,024 rows, 16
    above and for the bf16 chains."""
    cases = [  # (S, D, Z, n_enc, n_dec, dtype, extra, chain, dw, rows at B = 32 / 2048)
        (10, 3, 8, 4, 4, "fp32", {}, "f32", "f32", (4, 16)),                                # cfg1: the reference's own
        (100, 6, 8, 4, 4, "bf16", {}, "ring", "fast", (16, 16)),                             # cfg2 / cfg3 per rank
        (100, 6, 8, 4, 4, "bf16", dict(n_classes=4, class_dim=16), "ring", "cls", (16, 16)),  # cfg4
        (200, 6, 512, 8, 8, "bf16", {}, "wide", "wide", (16, 16)),                           # cfg5 bf16
        (200, 6, 512, 8, 8, "fp8", {}, "wide", "wide", (16, 16)),                            # cfg5 fp8
    ]
    for S, D, Z, ne, nd, dtype, extra, chain, dw, rows in cases:
        m = cvae.ConditionalTrajectoryVAE(S, D, Z, 128, ne, nd, **extra)
        e = m.attach(dtype=dtype, max_batch=2048, device="cuda:0")
        assert (e.train_kernel, e.dw_kernel) == (chain, dw), (S, D, Z, dtype, extra, e.train_kernel, e.dw_kernel)
        assert (e.chain_rows(32), e.chain_rows(2048)) == rows, (S, D, Z, dtype, e.chain_rows(32), e.chain_rows(2048))
        e.close()
