"""MI355X-native conditional trajectory VAE training path (yslf2035/Defensive-Model-VAE, Training_VAE.py).

Public API mirrors the reference module (Training_VAE.py):
  ConditionalTrajectoryVAE, conditional_vae_loss, TrajectoryDataset
plus the device engine (CVAEEngine: fused train step over the C-ABI in include/cvae.h),
the reference-shaped train loop (cvae_amd.train), data parallelism (cvae_amd.dist) and
trajectory generation (cvae_amd.tools, Tools.py:18-65).
"""
from .engine import CVAEEngine, config_info  # noqa: F401
from .model import ConditionalTrajectoryVAE, TrajectoryDataset, conditional_vae_loss  # noqa: F401
from .tools import generate_trajectories, load_model_and_generate_trajectory  # noqa: F401

__all__ = ["CVAEEngine", "ConditionalTrajectoryVAE", "TrajectoryDataset", "conditional_vae_loss", "config_info",
           "generate_trajectories", "load_model_and_generate_trajectory"]
