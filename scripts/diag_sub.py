"""GPU box, CVAE_DIAG_SUB build only: per-step sub-phase cycles (s_memtime) per wave of block 0."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "defensive-model-vae_amd")]
from cvae_amd import ConditionalTrajectoryVAE  # noqa: E402
from cvae_amd._lib import lib  # noqa: E402

B = 1024
torch.manual_seed(0)
m = ConditionalTrajectoryVAE(100, 6, 8)
eng = m.attach(dtype="bf16", max_batch=B)
x = eng.as_input(torch.randn(B, 100, 6))
L = lib()
L.cvae_diag_set_sub.argtypes = [C.c_void_p]
nb = (B + 31) // 32 * 32 // 16  # row-chain grid at R=16 (the kernel writes [block][wave][step][5])
NW = int(os.environ.get("NW", "8"))
buf = torch.zeros(nb * NW * 32 * 5, dtype=torch.int64, device="cuda")
L.cvae_diag_set_sub(C.c_void_p(buf.data_ptr()))
for _ in range(20):
    eng.train_step(x)
torch.cuda.synchronize()
st = buf.view(nb, NW, 32, 5).cpu().numpy().astype(np.int64)
blk = int(os.environ.get("BLK", "5"))
print("cycles (s_memtime) per step for block", blk, ": [entry->wait, wait->mfma, mfma->epi, epi->barrier, barrier->next entry]")
for si in range(20):
    row = []
    for w in range(NW):
        t = st[blk, w, si]
        nxt = st[blk, w, si + 1, 0] if si + 1 < 32 else 0
        if t[0] == 0:
            row.append("   -   ")
            continue
        d = [t[1] - t[0] if t[1] else -1, t[2] - t[1] if t[2] and t[1] else -1, t[3] - t[2] if t[3] and t[2] else -1,
             t[4] - (t[3] if t[3] else t[0]), (nxt - t[4]) if nxt else -1]
        row.append("/".join(str(int(v)) for v in d))
    print(f"step {si:2d}: " + "  ".join(f"w{w}:{r:>28s}" for w, r in enumerate(row)))
