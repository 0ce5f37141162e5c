"""Trajectory generation for the downstream callers (Tools.py:18-65 load_model_and_generate_trajectory).

Same signature, RNG use and return value as the reference function: a fresh module's init draws,
then z = torch.randn(1, latent_dim), both from the global CPU generator; h_c = condition_encoder([start_x, start_y]), the decoder's relative
trajectory [t, dx, dy] shifted by the start point, returned as a (seq_len, dim) numpy array.  The
decode runs on the MI355X through the C-ABI (cvae_decode, condition encoder fused); ``device``
selects the GPU ('cuda:N'); there is no CPU compute path, so 'cpu' (the reference's default) runs
on cuda:0 as well — the result is a host array either way.

The reference re-reads the checkpoint on every call (one call per MPC run, Distribution.py:73);
here the attached model is cached per (path, mtime, shape), so repeated calls cost one decode.
For many trajectories at once use ``generate_trajectories`` (one batched decode).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .model import ConditionalTrajectoryVAE

_CACHE: dict = {}


def _gpu(device):
    d = torch.device(device) if device is not None else torch.device("cuda", 0)
    return d if d.type == "cuda" else torch.device("cuda", 0)


def load_model(model_path, seq_len, dim, latent_dim, hidden_dim=128, device=None, max_batch=1024):
    """The checkpoint (24-key state_dict, Training_VAE.py:393) on the GPU, attached (fp32), cached."""
    dev = _gpu(device)
    key = (os.path.abspath(model_path), os.path.getmtime(model_path), seq_len, dim, latent_dim, hidden_dim,
           str(dev), max_batch)
    m = _CACHE.get(key)
    if m is None:
        with torch.random.fork_rng(devices=[]):  # loading leaves the caller's RNG stream untouched
            m = ConditionalTrajectoryVAE(seq_len, dim, latent_dim, hidden_dim)
        m.load_state_dict(torch.load(model_path, map_location="cpu", weights_only=True))
        m.attach(dtype="fp32", max_batch=max_batch, device=dev)
        _CACHE.clear()  # one model resident at a time
        _CACHE[key] = m
    return m


def load_model_and_generate_trajectory(model_path, start_x, start_y, seq_len=12, dim=3, latent_dim=8, device="cpu"):
    """Tools.py:18-65: one trajectory from the start point, (seq_len, dim) float32, absolute x/y."""
    m = load_model(model_path, seq_len, dim, latent_dim, device=device)
    # Tools.py:38 builds a fresh module before drawing z (:45) and its init draws from the global
    # CPU generator: build (and drop) one too, so z is the reference's z for the same seed
    ConditionalTrajectoryVAE(seq_len, dim, latent_dim)
    z = torch.randn(1, latent_dim)
    start = np.array([start_x, start_y], np.float32).reshape(1, 2)
    _, ab = m.generate(start, z=z)
    return ab[0].cpu().numpy()


def generate_trajectories(model_path, start_points, seq_len=12, dim=3, latent_dim=8, z=None, device=None):
    """Batched form: start_points (N, 2) → (N, seq_len, dim) absolute trajectories, z ~ N(0, I)
    (global CPU generator, drawn as one (N, latent_dim) tensor) unless given."""
    st = np.asarray(start_points, np.float32).reshape(-1, 2)
    m = load_model(model_path, seq_len, dim, latent_dim, device=device, max_batch=max(1024, st.shape[0]))
    if z is None:
        z = torch.randn(st.shape[0], latent_dim)
    _, ab = m.generate(st, z=z)
    return ab.cpu().numpy()
