"""Generate the golden vectors that pin the oracle to the reference.

TEST INFRASTRUCTURE — this script is the only file in the repo that imports the
reference (``/root/reference``, read-only).  It drives the reference's own
functions directly and writes small ``.npz`` fixtures next to itself:

* ``sce_fixed.npz``   — the shipped ``vae_offset_sce{1..4}_cond_ld8_epoch3000.pth``
  checkpoints evaluated on their own datasets (Training_VAE.py:180-268).  sce1
  is stored in full (weights, inputs, recon/mu/logvar/h_c at z=mu and at a
  seeded eps, the 5 losses, all 24 gradients); sce2-4 keep the 5 losses.
* ``step1_h16.npz``   — a tiny config (S=10, D=3, Z=8, H=16, B=8) seeded
  init, one fwd+bwd+Adam step exactly as Training_VAE.py:345-363.
* ``traj20_sce1.npz`` — the reference train loop (Training_VAE.py:326-370) on
  sce1 at batch 32 for 20 steps (10 epochs) from ``torch.manual_seed(0)``:
  per-step losses, the per-step eps and batch index orders the host RNG
  produced, initial and final parameters.
* ``cfg2_small.npz``  — the north-star shape (S=100, D=6, H=128, Z=8) at B=64
  with x ~ N(0,1) (generator seed 1234) and eps seed 4321: losses, per-tensor
  gradient norms and leading slices.

Run here (not on the GPU box):  ``python tests/golden/make_goldens.py``.
The reference never travels; only these fixtures do.
"""
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
W = dict(recon_weight=0.1, kld_weight=0.1, start_weight=1.0, time_weight=1.0)  # Training_VAE.py:300-306


def _import_reference():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import Tools  # noqa: F401  (Training_VAE.py:102 <-> Tools.py:14 import cycle: Tools first)
    import Training_VAE as tv
    return tv


def _state_np(model):
    return {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}


def _rel(batch):
    # Training_VAE.py:345-348
    start = batch[:, 0, 1:3]
    rel = batch.clone()
    rel[:, :, 1:3] = rel[:, :, 1:3] - start.unsqueeze(1)
    return rel, start


def _fwd_fixed_eps(tv, model, rel, start, eps):
    mu, logvar, hc = model.encode(rel, start)
    z = mu + eps * torch.exp(0.5 * logvar)          # Training_VAE.py:204-206 with eps given
    recon = model.decode(z, hc)
    return recon, mu, logvar, hc


def make_sce_fixed(tv, out):
    res = {}
    for sce in (1, 2, 3, 4):
        data = tv.TrajectoryDataset(f"{REF}/training/DefensiveDataProcessed/trajectory_sce{sce}_cond.npy")
        batch = torch.from_numpy(data.data)
        sd = torch.load(f"{REF}/training/models/vae_offset_sce{sce}_cond_ld8_epoch3000.pth",
                        map_location="cpu", weights_only=True)
        model = tv.ConditionalTrajectoryVAE(10, 3, 8)
        model.load_state_dict(sd)
        rel, start = _rel(batch)
        with torch.no_grad():
            mu, logvar, hc = model.encode(rel, start)
            recon = model.decode(mu, hc)
            losses = tv.conditional_vae_loss(recon, rel, mu, logvar, hc, **W)
        res[f"sce{sce}_losses_zmu"] = np.array([float(x) for x in losses], np.float64)
        if sce == 1:
            for k, v in sd.items():
                res["w/" + k] = v.numpy()
            res["sce1_x"] = data.data
            res["sce1_recon_zmu"] = recon.numpy()
            res["sce1_mu"] = mu.numpy()
            res["sce1_logvar"] = logvar.numpy()
            res["sce1_hc"] = hc.numpy()
            g = torch.Generator().manual_seed(4321)
            eps = torch.randn(batch.shape[0], 8, generator=g)
            model.zero_grad()
            recon, mu, logvar, hc = _fwd_fixed_eps(tv, model, rel, start, eps)
            losses = tv.conditional_vae_loss(recon, rel, mu, logvar, hc, **W)
            losses[0].backward()
            res["sce1_eps"] = eps.numpy()
            res["sce1_recon_eps"] = recon.detach().numpy()
            res["sce1_losses_eps"] = np.array([float(x) for x in losses], np.float64)
            for k, p in model.named_parameters():
                res["g/" + k] = p.grad.numpy().copy()
    np.savez_compressed(out, **res)


def make_step1_h16(tv, out):
    torch.manual_seed(0)
    model = tv.ConditionalTrajectoryVAE(10, 3, 8, hidden_dim=16)
    init = _state_np(model)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    data = tv.TrajectoryDataset(f"{REF}/training/DefensiveDataProcessed/trajectory_sce1_cond.npy")
    batch = torch.from_numpy(data.data[:8].copy())
    rel, start = _rel(batch)
    eps = torch.randn(8, 8, generator=torch.Generator().manual_seed(7))
    opt.zero_grad()
    recon, mu, logvar, hc = _fwd_fixed_eps(tv, model, rel, start, eps)
    losses = tv.conditional_vae_loss(recon, rel, mu, logvar, hc, **W)
    losses[0].backward()
    grads = {k: p.grad.numpy().copy() for k, p in model.named_parameters()}
    opt.step()
    res = {"x": batch.numpy(), "eps": eps.numpy(), "recon": recon.detach().numpy(),
           "mu": mu.detach().numpy(), "logvar": logvar.detach().numpy(), "hc": hc.detach().numpy(),
           "losses": np.array([float(x) for x in losses], np.float64)}
    for k, v in init.items():
        res["init/" + k] = v
    for k, v in grads.items():
        res["g/" + k] = v
    for k, v in _state_np(model).items():
        res["post/" + k] = v
    np.savez_compressed(out, **res)


def make_traj20(tv, out, steps=20, seed=0, batch_size=32):
    from torch.utils.data import DataLoader
    captured = []
    orig = torch.randn_like

    def rec(t, *a, **k):
        o = orig(t, *a, **k)
        captured.append(o.detach().clone())
        return o

    torch.manual_seed(seed)
    path = f"{REF}/training/DefensiveDataProcessed/trajectory_sce1_cond.npy"
    dataset = tv.TrajectoryDataset(path)                                # :326
    loader = DataLoader(dataset, batch_size=batch_size, shuffle=True)   # :327
    model = tv.ConditionalTrajectoryVAE(10, 3, 8)                       # :331
    init = _state_np(model)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)                 # :332
    model.train()
    losses, orders = [], []
    torch.randn_like = rec
    try:
        n = 0
        while n < steps:
            for batch in loader:                                        # :340
                rel, start = _rel(batch)
                opt.zero_grad()
                recon, mu, logvar, hc = model(rel, start)
                ls = tv.conditional_vae_loss(recon, rel, mu, logvar, hc, **W)
                ls[0].backward()
                opt.step()
                losses.append([float(x) for x in ls])
                # recover the sampled indices by row matching (rows are unique)
                idx = [int(np.nonzero(np.all(dataset.data == r, axis=(1, 2)))[0][0]) for r in batch.numpy()]
                orders.append(idx)
                n += 1
                if n == steps:
                    break
    finally:
        torch.randn_like = orig
    res = {"losses": np.array(losses, np.float64), "batch_size": np.int64(batch_size), "seed": np.int64(seed)}
    res["eps"] = np.concatenate([c.numpy() for c in captured], 0)
    res["eps_rows"] = np.array([c.shape[0] for c in captured], np.int64)
    res["order"] = np.array([i for o in orders for i in o], np.int64)
    for k, v in init.items():  # init is regenerated from the seed; keep a checksum to pin it
        res["init_sum/" + k] = np.float64(v.astype(np.float64).sum())
        res["init_head/" + k] = v.reshape(-1)[:8].copy()
    for k, v in _state_np(model).items():
        res["final/" + k] = v
    np.savez_compressed(out, **res)


def make_cfg2_small(tv, out, B=64):
    torch.manual_seed(0)
    model = tv.ConditionalTrajectoryVAE(100, 6, 8)
    x = torch.randn(B, 100, 6, generator=torch.Generator().manual_seed(1234))
    eps = torch.randn(B, 8, generator=torch.Generator().manual_seed(4321))
    rel, start = _rel(x)
    recon, mu, logvar, hc = _fwd_fixed_eps(tv, model, rel, start, eps)
    ls = tv.conditional_vae_loss(recon, rel, mu, logvar, hc, **W)
    ls[0].backward()
    res = {"losses": np.array([float(v) for v in ls], np.float64), "x_head": x.reshape(-1)[:16].numpy(),
           "recon_row0": recon[0].detach().numpy(), "mu": mu.detach().numpy(), "logvar": logvar.detach().numpy()}
    for k, p in model.named_parameters():
        res["gnorm/" + k] = np.float64(p.grad.double().norm())
        res["ghead/" + k] = p.grad.reshape(-1)[:32].numpy().copy()
        res["phead/" + k] = p.detach().reshape(-1)[:32].numpy().copy()
    np.savez_compressed(out, **res)


if __name__ == "__main__":
    tv = _import_reference()
    torch.set_num_threads(1)
    make_sce_fixed(tv, os.path.join(HERE, "sce_fixed.npz"))
    make_step1_h16(tv, os.path.join(HERE, "step1_h16.npz"))
    make_traj20(tv, os.path.join(HERE, "traj20_sce1.npz"))
    make_cfg2_small(tv, os.path.join(HERE, "cfg2_small.npz"))
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
