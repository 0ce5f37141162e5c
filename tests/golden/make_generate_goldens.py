"""Golden vectors for single-trajectory generation (Tools.load_model_and_generate_trajectory,
Tools.py:18-65) — TEST INFRASTRUCTURE, run here (not on the GPU box).

Calls the reference function itself on the shipped sce1 checkpoint
(training/models/vae_offset_sce1_cond_ld8_epoch3000.pth, whose 24 tensors are already stored in
sce_fixed.npz as ``w/*``) for a few start points, each after ``torch.manual_seed(seed)`` (the
function builds a fresh ConditionalTrajectoryVAE — whose init draws from the global CPU
generator — and then draws z = torch.randn(1, latent_dim) from it), and writes
``generate_sce1.npz``: seeds, start points, the z each call drew, and the returned (seq_len, 3)
absolute trajectories.  Run: ``python tests/golden/make_generate_goldens.py``.
"""
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
CKPT = os.path.join(REF, "training/models/vae_offset_sce1_cond_ld8_epoch3000.pth")


def main():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import Tools  # noqa: F401  (Training_VAE.py:102 <-> Tools.py:14 import cycle: Tools first)
    import Training_VAE

    starts = np.array([[0.0, 0.0], [152.5, -37.25], [-20.0, 88.0], [3.5, 4.25]], np.float32)
    seeds = np.array([0, 1, 7, 1234])
    zs, outs = [], []
    for s, (sx, sy) in zip(seeds, starts):
        torch.manual_seed(int(s))  # the z the call below draws: after the module's own init draws
        Training_VAE.ConditionalTrajectoryVAE(10, 3, 8)
        zs.append(torch.randn(1, 8).numpy()[0])
        torch.manual_seed(int(s))
        outs.append(Tools.load_model_and_generate_trajectory(CKPT, float(sx), float(sy), seq_len=10, dim=3,
                                                             latent_dim=8, device="cpu"))
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "generate_sce1.npz")
    np.savez(out, seeds=seeds, starts=starts, z=np.stack(zs).astype(np.float32),
             traj=np.stack(outs).astype(np.float32))
    print("wrote", out)


if __name__ == "__main__":
    main()
