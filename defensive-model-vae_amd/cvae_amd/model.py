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

Two ways to train:

* the fused step — ``cvae_amd.train`` / ``CVAEEngine.train_step`` (forward, loss, backward and
  Adam in two kernels, no autograd);
* the reference's own loop, unchanged (Training_VAE.py:338-363): ``model(batch_rel, start)``
  returns autograd-tracked outputs (``_ForwardFn``: cvae_forward, backward = cvae_backward),
  ``conditional_vae_loss`` is differentiable (``_LossFn``: cvae_loss / cvae_loss_backward), so
  ``loss.backward()`` fills ``p.grad`` through the HIP kernels and any torch optimizer over
  ``model.parameters()`` steps them; the engine repacks its operand copies when it sees the
  parameters' version counters move.
"""
from __future__ import annotations

import ctypes as C
import weakref

import numpy as np
import torch
import torch.nn as nn

from ._lib import CvaeLossWeights, check, lib, ptr
from .engine import CVAEEngine


class _ForwardFn(torch.autograd.Function):
    """model.forward as one autograd node: outputs (recon, mu, logvar, h_c) of cvae_forward; the
    backward recomputes the same forward (same eps / Philox offset) and back-propagates the four
    output gradients to every parameter (cvae_backward)."""

    @staticmethod
    def forward(ctx, eng, x, start, eps, offset, classes, *params):
        recon, mu, lv, hc = eng.forward(x, start=start, eps=eps, offset=offset, classes=classes)
        ctx.eng, ctx.offset = eng, offset
        ctx.save_for_backward(x, start, eps, classes)
        return recon, mu, lv, hc

    @staticmethod
    def backward(ctx, d_recon, d_mu, d_lv, d_hc):
        x, start, eps, classes = ctx.saved_tensors
        eng = ctx.eng
        flat = eng.backward(x, start, eps, ctx.offset, d_recon, d_mu, d_lv, d_hc, classes=classes)
        return (None, None, None, None, None, None, *eng.views(flat))


class _LossFn(torch.autograd.Function):
    """conditional_vae_loss as one autograd node: the 5 losses (cvae_loss); backward
    cvae_loss_backward (dL/drecon, dL/dmu, dL/dlogvar from the 5 upstream gradients)."""

    @staticmethod
    def forward(ctx, recon, x, mu, logvar, weights):
        B, S, D = recon.shape
        Z = mu.shape[1]
        dev = recon.device
        out = torch.empty(5, device=dev, dtype=torch.float32)
        ws = torch.empty(8 * ((B + 31) // 32), device=dev, dtype=torch.float32)
        w = CvaeLossWeights(*weights)
        with torch.cuda.device(dev):
            check(lib().cvae_loss(ptr(recon), ptr(x), ptr(mu), ptr(logvar), B, S, D, Z, C.byref(w), ptr(out), ptr(ws),
                                  C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "cvae_loss")
        ctx.weights = weights
        ctx.save_for_backward(recon, x, mu, logvar)
        return out

    @staticmethod
    def backward(ctx, g):
        recon, x, mu, logvar = ctx.saved_tensors
        B, S, D = recon.shape
        Z = mu.shape[1]
        dev = recon.device
        g = g.to(device=dev, dtype=torch.float32).contiguous()
        d_recon, d_mu, d_lv = torch.empty_like(recon), torch.empty_like(mu), torch.empty_like(logvar)
        w = CvaeLossWeights(*ctx.weights)
        with torch.cuda.device(dev):
            check(lib().cvae_loss_backward(ptr(recon), ptr(x), ptr(mu), ptr(logvar), B, S, D, Z, C.byref(w), ptr(g),
                                           ptr(d_recon), ptr(d_mu), ptr(d_lv),
                                           C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                  "cvae_loss_backward")
        return d_recon, None, d_mu, d_lv, None


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
    """Training_VAE.py:118-226.  n_enc/n_dec generalise the 4+4 depth (BASELINE cfg5).

    n_classes > 0 (BASELINE cfg4, a build-side extension the reference does not have): a scenario
    class embedding ``class_embedding = nn.Embedding(n_classes, class_dim)`` whose row e joins both
    concatenations beside h_c — fc input [h_traj ‖ h_c ‖ e] (:193) and decoder input
    [z ‖ h_c ‖ e] (:214).  It is registered last, so the reference's 24 keys and init stream come
    first; its parity is pinned to the extended oracle, not to the reference."""

    def __init__(self, seq_len, dim, latent_dim, hidden_dim=128, n_enc=4, n_dec=4, n_classes=0, class_dim=16):
        super().__init__()
        self.seq_len, self.dim, self.latent_dim, self.hidden_dim = seq_len, dim, latent_dim, hidden_dim
        self.n_enc, self.n_dec = n_enc, n_dec
        self.n_classes, self.class_dim = int(n_classes), (int(class_dim) if n_classes else 0)
        H, I, Z, E = hidden_dim, seq_len * dim, latent_dim, self.class_dim
        # module order = reference order (init RNG stream and state_dict keys)
        self.condition_encoder = _ConditionEncoder(nn.Linear(2, H), nn.ReLU(), nn.Linear(H, H), nn.ReLU())
        enc = [nn.Flatten()]
        for i in range(n_enc):
            enc += [nn.Linear(I if i == 0 else H, H), nn.ReLU()]
        self.encoder = nn.Sequential(*enc)
        self.fc_mu = nn.Linear(H + H + E, Z)
        self.fc_logvar = nn.Linear(H + H + E, Z)
        dec = []
        for i in range(n_dec - 1):
            dec += [nn.Linear(Z + H + E if i == 0 else H, H), nn.ReLU()]
        dec += [nn.Linear(H, I), nn.Unflatten(1, (seq_len, dim))]
        self.decoder = nn.Sequential(*dec)
        if self.n_classes:
            self.class_embedding = nn.Embedding(self.n_classes, E)
        self.__dict__["_engine"] = None
        self.condition_encoder.__dict__["_owner"] = weakref.ref(self)

    # ------------------------------------------------------------------ device binding
    def attach(self, dtype="fp32", max_batch=1024, device=None, seed=0):
        """Create the HIP engine and make the parameters views of its flat buffer."""
        eng = CVAEEngine(self.seq_len, self.dim, self.latent_dim, self.hidden_dim, self.n_enc, self.n_dec,
                         dtype=dtype, max_batch=max_batch, device=device, seed=seed, n_classes=self.n_classes,
                         class_dim=self.class_dim)
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

    def encode(self, x, start_points, classes=None):  # :180-197
        _, mu, logvar, hc = _need(self).forward(x, start=start_points, outputs=("mu", "logvar", "hc"),
                                                classes=classes)
        return mu, logvar, hc

    def reparameterize(self, mu, logvar):  # :199-206 (elementwise helper; the training path fuses it)
        std = torch.exp(0.5 * logvar)
        return mu + torch.randn_like(std) * std

    def decode(self, z, condition, classes=None):  # :208-215 — condition = h_c features
        return _need(self).decode(z, hc=condition, classes=classes)

    def forward(self, x, start_points, eps=None, classes=None):  # :217-226 (x relative, start absolute)
        """model(batch_rel, start_points) → (recon, mu, logvar, h_c), autograd-tracked.

        eps (the reparameterisation noise, :205): None draws ``torch.randn(B, Z)`` from the global
        CPU generator — the stream the reference's CPU run consumes (Training_VAE.py:282 runs on
        'cpu'), so a seeded loop replays it; a (B, Z) tensor is used as given; "philox" draws it
        in-kernel (Philox at the engine's next offset)."""
        eng = _need(self)
        B = x.shape[0]
        offset = 0
        if eps is None:
            eps = torch.randn(B, self.latent_dim)
        if isinstance(eps, str):
            if eps != "philox":
                raise ValueError("eps must be None, a (B, Z) tensor or 'philox'")
            eps, offset = None, eng.rng_offset
            eng.rng_offset = offset + 1
        else:
            eps = torch.as_tensor(eps).to(device=eng.device, dtype=torch.float32).contiguous()
        x = eng.as_input(x, keep_f32=True).detach()
        start = torch.as_tensor(start_points).to(device=eng.device, dtype=torch.float32).contiguous().detach()
        cl = eng._classes(classes, B)
        return _ForwardFn.apply(eng, x, start, eps, offset, cl, *self.parameters())

    def generate(self, start_points, z=None, generator=None, classes=None):
        """Batched sampling (Tools.py:18-65): z ~ N(0,I); returns (relative, absolute) trajectories."""
        eng = _need(self)
        st = torch.as_tensor(start_points, dtype=torch.float32, device=eng.device).reshape(-1, 2)
        if z is None:
            z = torch.randn(st.shape[0], self.latent_dim, device=eng.device, generator=generator)
        rel = eng.decode(z, start=st, classes=classes)
        ab = rel.clone()
        ab[:, :, 1:3] += st[:, None, :]
        return rel, ab


def conditional_vae_loss(recon_x, x, mu, logvar, condition=None, recon_weight=0.1, kld_weight=0.1,
                         start_weight=1.0, time_weight=0.5):
    """Training_VAE.py:229-268 (5-tuple, same defaults), differentiable: the HIP kernels cvae_loss
    (forward) and cvae_loss_backward (autograd).  Device tensors only."""
    if not recon_x.is_cuda:
        raise RuntimeError("conditional_vae_loss runs on the HIP device (cvae_loss); got a CPU tensor")
    dev = recon_x.device
    f = lambda t: t.to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
    w = (float(recon_weight), float(kld_weight), float(start_weight), float(time_weight))
    out = _LossFn.apply(f(recon_x), f(x).detach(), f(mu), f(logvar), w)
    return tuple(out[i] for i in range(5))


class TrajectoryDataset(torch.utils.data.Dataset):
    """Training_VAE.py:105-115: (N,S,D) npy → float32."""

    def __init__(self, data_path):
        self.data = np.load(data_path).astype(np.float32)

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        return self.data[idx]
