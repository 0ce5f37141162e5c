"""The wide chain's eps drawn ahead (BASELINE cfg5, wchain::EpsPre): the dW launch of a Philox step
draws the next step's eps in blocks behind its tiles, and the next row chain takes them when the key
{offset, eps_row0, seed, rows} names its own draw (Training_VAE.py:199-206 reparameterize; the
values are the same Philox4x32-10 normals either way).  Needs the MI355X.

Bit-equality against a handle created with CVAE_EPS_AHEAD=0 (every chain draws its own): the first
step (no key yet), full steps (key hit), a smaller batch followed by a larger one (the rows past the
drawn ones draw in the chain), a host-eps step in between (no draw ahead), a counter rewind (the key
names an offset the chain does not use), and the split path (forward_backward + adam_step)."""
import pytest
import torch

from oracle.cvae_oracle import OracleCVAE

pytestmark = pytest.mark.gpu
WIDE = dict(S=200, D=6, Z=512, n_enc=8, n_dec=8)


@pytest.fixture(scope="module")
def cvae():
    import cvae_amd
    assert torch.cuda.is_available()
    return cvae_amd


def _engines(cvae, monkeypatch, dtype):
    c = WIDE
    torch.manual_seed(2)
    ref = OracleCVAE(c["S"], c["D"], c["Z"], 128, c["n_enc"], c["n_dec"])
    out = []
    for ahead in ("1", "0"):
        monkeypatch.setenv("CVAE_EPS_AHEAD", ahead)
        m = cvae.ConditionalTrajectoryVAE(c["S"], c["D"], c["Z"], 128, c["n_enc"], c["n_dec"])
        m.load_state_dict(ref.state_dict())
        e = m.attach(dtype=dtype, max_batch=256, device="cuda:0", seed=9)
        monkeypatch.delenv("CVAE_EPS_AHEAD")
        assert e.train_kernel == "wide" and e.dw_kernel == "wide"
        out.append(e)
    return out


def _same(e1, e2):
    torch.cuda.synchronize()
    assert torch.equal(e1.params, e2.params)
    assert torch.equal(e1.m, e2.m) and torch.equal(e1.v, e2.v)
    assert torch.equal(e1.loss, e2.loss)
    assert torch.equal(e1.counters, e2.counters)


@pytest.mark.parametrize("dtype", ["fp8", "bf16"])
def test_eps_ahead_equals_in_chain_draws(cvae, monkeypatch, dtype):
    e1, e2 = _engines(cvae, monkeypatch, dtype)
    g = torch.Generator().manual_seed(17)
    data = torch.randn(300, 200, 6, generator=g)
    x1, x2 = e1.as_input(data), e2.as_input(data)
    idx = torch.randperm(300, generator=g)[:256].cuda()
    for b in (256, 256, 256, 100, 256):  # first step: no key; then hits; 100 rows: a 128-row draw
        for e, x in ((e1, x1), (e2, x2)):
            e.train_step(x, idx=idx[:b])
        _same(e1, e2)
    eps = torch.randn(256, 512, generator=g)
    for e, x in ((e1, x1), (e2, x2)):  # host eps: no draw ahead; the next Philox step draws itself
        e.train_step(x, idx=idx, eps=eps)
        e.train_step(x, idx=idx)
        e.train_step(x, idx=idx)
    _same(e1, e2)
    for e in (e1, e2):  # rewind the Philox offset: the key no longer names the chain's draw
        e.counters[0].sub_(2)
    for e, x in ((e1, x1), (e2, x2)):
        e.train_step(x, idx=idx)
        e.train_step(x, idx=idx)
    _same(e1, e2)
    for e, x in ((e1, x1), (e2, x2)):  # the split path: fwd/bwd (draws ahead too), then Adam
        e.forward_backward(x, idx=idx)
        e.adam_step(1.0)
        e.forward_backward(x, idx=idx)
    torch.cuda.synchronize()
    assert torch.equal(e1.grads, e2.grads)
    _same(e1, e2)


def test_eps_ahead_train_steps_and_epochs(cvae, monkeypatch):
    """The multi-step entry points (cvae_train_steps: one C call; cvae_train_epochs: shuffled
    epochs, a ragged last batch) with the draw ahead between every two steps."""
    e1, e2 = _engines(cvae, monkeypatch, "fp8")
    g = torch.Generator().manual_seed(23)
    data = torch.randn(300, 200, 6, generator=g)
    x1, x2 = e1.as_input(data), e2.as_input(data)
    for e, x in ((e1, x1), (e2, x2)):
        e.train_steps(x, 5, batch=256)
    _same(e1, e2)
    perms = torch.stack([torch.randperm(300, generator=g) for _ in range(3)]).cuda()
    for e, x in ((e1, x1), (e2, x2)):
        acc = e.train_epochs(x, perms, 128)  # 3 epochs of 128, 128, 44 rows
    _same(e1, e2)
