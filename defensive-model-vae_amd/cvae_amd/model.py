"""Reference-compatible API of Training_VAE.py, computed by the HIP kernels.

* ``ConditionalTrajectoryVAE(seq_len, dim, latent_dim, hidden_dim=128)`` —
  Training_VAE.py:118-226.  Same constructor, same submodule names and module
  order (so ``torch.manual_seed`` init and the 24-key state_dict are identical
  and ``Tools.py:39-41`` ``load_state_dict`` works unchanged).  After
  ``attach()`` the parameters are views of the engine's flat fp32 buffer and
  ``encode/decode/forward/condition_encoder`` run the C-ABI kernels.  There is
  no torch-compute fallback: computing on a module that is not attached to a
  HIP device raises.
* ``conditional_vae_loss(...)`` — Training_VAE.py:229-268 via ``cvae_loss``.
* ``TrajectoryDataset(path)`` — Training_VAE.py:105-115.

Training goes through ``cvae_amd.train`` / ``CVAEEngine.train_step`` (the fused
step); the module's outputs carry no autograd graph.
"""
from __future__ import annotations

import ctypes as C
import weakref

import numpy as np
import torch
import torch.nn as nn

from ._lib import CvaeLossWeights, check, lib, ptr
from .engine import CVAEEngine


def _need(model):
    eng = getattr(model, "_engine", None)
    if eng is None:
        raise RuntimeError("ConditionalTrajectoryVAE computes on the HIP device: call model.attach() "
                           "(MI355X) first — there is no CPU/torch fallback")
    return eng


class _ConditionEncoder(nn.Sequential):
    """condition_encoder (Training_VAE.py:132-137); forward runs cvae_condition."""

    def forward(self, start):
        owner = self.__dict__.get("_owner")
        model = owner() if owner is not None else None
        if model is None:
            raise RuntimeError("condition_encoder is bound to a ConditionalTrajectoryVAE; call model.attach()")
        return _need(model).condition(start)


class ConditionalTrajectoryVAE(nn.Module):
    def __init__(self, seq_len, dim, latent_dim, hidden_dim=128, n_enc=4, n_dec=4):
        super().__init__()
        self.seq_len, self.dim, self.latent_dim, self.hidden_dim = seq_len, dim, latent_dim, hidden_dim
        self.n_enc, self.n_dec = n_enc, n_dec
        H, I, Z = hidden_dim, seq_len * dim, latent_dim
        # module order = reference order (init RNG stream and state_dict keys)
        self.condition_encoder = _ConditionEncoder(nn.Linear(2, H), nn.ReLU(), nn.Linear(H, H), nn.ReLU())
        enc = [nn.Flatten()]
        for i in range(n_enc):
            enc += [nn.Linear(I if i == 0 else H, H), nn.ReLU()]
        self.encoder = nn.Sequential(*enc)
        self.fc_mu = nn.Linear(H + H, Z)
        self.fc_logvar = nn.Linear(H + H, Z)
        dec = []
        for i in range(n_dec - 1):
            dec += [nn.Linear(Z + H if i == 0 else H, H), nn.ReLU()]
        dec += [nn.Linear(H, I), nn.Unflatten(1, (seq_len, dim))]
        self.decoder = nn.Sequential(*dec)
        self.__dict__["_engine"] = None
        self.condition_encoder.__dict__["_owner"] = weakref.ref(self)

    # ------------------------------------------------------------------ device binding
    def attach(self, dtype="fp32", max_batch=1024, device=None, seed=0):
        """Create the HIP engine and make the parameters views of its flat buffer."""
        eng = CVAEEngine(self.seq_len, self.dim, self.latent_dim, self.hidden_dim, self.n_enc, self.n_dec,
                         dtype=dtype, max_batch=max_batch, device=device, seed=seed)
        eng.bind(self)
        self.__dict__["_engine"] = eng
        return eng

    @property
    def engine(self):
        return _need(self)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        if self.__dict__.get("_engine") is not None:
            if assign:
                raise RuntimeError("assign=True would detach parameters from the engine buffer")
            self._engine.pack()
        return res

    # ------------------------------------------------------------------ reference methods
    def get_start_points(self, x):  # Training_VAE.py:169-178
        return x[:, 0, 1:3]

    def encode(self, x, start_points):  # :180-197
        _, mu, logvar, hc = _need(self).forward(x, start=start_points, outputs=("mu", "logvar", "hc"))
        return mu, logvar, hc

    def reparameterize(self, mu, logvar):  # :199-206 (elementwise helper; the training path fuses it)
        std = torch.exp(0.5 * logvar)
        return mu + torch.randn_like(std) * std

    def decode(self, z, condition):  # :208-215 — condition = h_c features
        return _need(self).decode(z, hc=condition)

    def forward(self, x, start_points, eps=None):  # :217-226 (x relative, start absolute)
        return _need(self).forward(x, start=start_points, eps=eps)

    def generate(self, start_points, z=None, generator=None):
        """Batched sampling (Tools.py:18-65): z ~ N(0,I); returns (relative, absolute) trajectories."""
        eng = _need(self)
        st = torch.as_tensor(start_points, dtype=torch.float32, device=eng.device).reshape(-1, 2)
        if z is None:
            z = torch.randn(st.shape[0], self.latent_dim, device=eng.device, generator=generator)
        rel = eng.decode(z, start=st)
        ab = rel.clone()
        ab[:, :, 1:3] += st[:, None, :]
        return rel, ab


def conditional_vae_loss(recon_x, x, mu, logvar, condition=None, recon_weight=0.1, kld_weight=0.1,
                         start_weight=1.0, time_weight=0.5):
    """Training_VAE.py:229-268 (5-tuple, same defaults).  HIP kernel; device tensors only."""
    if not recon_x.is_cuda:
        raise RuntimeError("conditional_vae_loss runs on the HIP device (cvae_loss); got a CPU tensor")
    B, S, D = recon_x.shape
    Z = mu.shape[1]
    dev = recon_x.device
    f = lambda t: t.detach().to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
    r, xx, m, lv = f(recon_x), f(x), f(mu), f(logvar)
    out = torch.empty(5, device=dev, dtype=torch.float32)
    ws = torch.empty(8 * ((B + 31) // 32), device=dev, dtype=torch.float32)
    w = CvaeLossWeights(recon_weight, kld_weight, start_weight, time_weight)
    with torch.cuda.device(dev):
        check(lib().cvae_loss(ptr(r), ptr(xx), ptr(m), ptr(lv), B, S, D, Z, C.byref(w), ptr(out), ptr(ws),
                              C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "cvae_loss")
    return tuple(out[i] for i in range(5))


class TrajectoryDataset(torch.utils.data.Dataset):
    """Training_VAE.py:105-115: (N,S,D) npy → float32."""

    def __init__(self, data_path):
        self.data = np.load(data_path).astype(np.float32)

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        return self.data[idx]
