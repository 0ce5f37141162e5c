"""GPU box, diagnostic build only: per-phase time of the row-chain kernel from in-kernel stamps.

CVAE_LIB=build/diag/stamps.so python scripts/diag_stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "defensive-model-vae_amd")]
from cvae_amd import ConditionalTrajectoryVAE  # noqa: E402
from cvae_amd._lib import lib  # noqa: E402

B = int(os.environ.get("B", "1024"))
dtype = os.environ.get("DT", "bf16")
torch.manual_seed(0)
m = ConditionalTrajectoryVAE(100, 6, 8)
eng = m.attach(dtype=dtype, max_batch=B)
x = eng.as_input(torch.randn(B, 100, 6))
L = lib()
L.cvae_diag_set_stamps.argtypes = [C.c_void_p, C.c_void_p]
R = 16
nb = ((B + 31) // 32 * 32) // R
dbuf = torch.zeros(nb * 64, dtype=torch.int64, device="cuda")
L.cvae_diag_set_stamps(eng._h, C.c_void_p(dbuf.data_ptr()))
for _ in range(30):
    eng.train_step(x)
torch.cuda.synchronize()
st = dbuf.view(nb, 64).cpu().numpy().astype(np.int64)
k = int((st[0] > 0).sum())
d = np.diff(st[:, :k], axis=1) * 10  # ns
t0 = st[:, 0].min()
print(f"blocks={nb} stamps={k} kernel span={(st[:, k-1].max() - t0) * 10 / 1000:.2f} us; start skew={(st[:,0].max()-t0)*10/1000:.2f} us")
names = ["prologue", "xT copies+C0"] + [f"step{i}" for i in range(1, 64)]
for i in range(k - 1):
    print(f"{names[i]:>14s} {i:2d}: median {np.median(d[:, i]) / 1000:7.3f} us   max {d[:, i].max() / 1000:7.3f} us")
