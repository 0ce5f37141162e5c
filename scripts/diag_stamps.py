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
WIDE = os.environ.get("WIDE") == "1"  # BASELINE cfg5's shape (the wide chain)
F32 = os.environ.get("F32") == "1"    # the reference's own shape in fp32 (the fp32 ring chain)
if F32:
    dtype = "fp32"
    m = ConditionalTrajectoryVAE(10, 3, 8)
else:
    m = ConditionalTrajectoryVAE(200, 6, 512, 128, 8, 8) if WIDE else ConditionalTrajectoryVAE(100, 6, 8)
eng = m.attach(dtype=dtype, max_batch=B)
x = eng.as_input(torch.randn(B, 10, 3) * 5 if F32 else torch.randn(B, 200, 6) if WIDE else torch.randn(B, 100, 6))
L = lib()
L.cvae_diag_set_stamps.argtypes = [C.c_void_p, C.c_void_p]
L.cvae_diag_set_wstamps.argtypes = [C.c_void_p]
R = eng.chain_rows(B)  # rows per chain workgroup (the fp32 chain: 4 up to 1,024 rows)
nb = ((B + 31) // 32 * 32) // R
dbuf = torch.zeros(nb * 64, dtype=torch.int64, device="cuda")
NT = 4096
wbuf = torch.zeros(NT * 8, dtype=torch.int64, device="cuda")
for _ in range(30):
    eng.train_step(x)
torch.cuda.synchronize()
L.cvae_diag_set_stamps(eng._h, C.c_void_p(dbuf.data_ptr()))
L.cvae_diag_set_wstamps(C.c_void_p(wbuf.data_ptr()))
if os.environ.get("MODE") == "split":
    eng.forward_backward(x)  # the separate row-chain launch (fastchain_kernel) and dW launch
else:
    eng.train_step(x)  # the measured step: both kernels stamp their blocks
torch.cuda.synchronize()
L.cvae_diag_set_wstamps(C.c_void_p(0))
st = dbuf.view(nb, 64).cpu().numpy().astype(np.int64)
k = int((st[0] > 0).sum())
d = np.diff(st[:, :k], axis=1) * 10  # ns
t0 = st[:, 0].min()
print(f"blocks={nb} stamps={k} kernel span={(st[:, k-1].max() - t0) * 10 / 1000:.2f} us; start skew={(st[:,0].max()-t0)*10/1000:.2f} us")
names = ["prologue", "xT copies+C0"] + [f"step{i}" for i in range(1, 64)]
if WIDE:
    names = (["prologue", "C0|E0", "C1|E1"] + [f"E{i}" for i in range(2, 8)] + ["FC", "D0"]
             + [f"D{i}" for i in range(1, 7)] + ["D7+loss", "fixup", "D7b"] + [f"D{i}b" for i in range(6, 0, -1)]
             + ["D0b", "FCb"] + [f"E{i}b" for i in range(7, 1, -1)] + ["E1b|C1b", "partials"])
    if os.environ.get("SUB") == "1":  # CVAE_DIAG_STAMPS=2: stamps inside some steps
        names = (["pro:issue", "pro:transform", "pro:bar", "C0+copies", "E0 gemm", "E0 epi", "C1|E1"]
                 + [f"E{i}" for i in range(2, 8)] + ["FC", "D0"] + [f"D{i}" for i in range(1, 7)]
                 + ["D7+loss", "fixup", "D7b"] + [f"D{i}b" for i in range(6, 0, -1)]
                 + ["D0b", "FCb gemm", "FCb epi"] + [f"E{i}b" for i in range(7, 1, -1)] + ["E1b|C1b", "partials"])
        if os.environ.get("DT") == "fp8":  # the MX dX steps stamp the end of their operand conversion
            for n, m in (("D7b", ["D7b mx cvt", "D7b"]), ("D0b", ["D0b mx cvt", "D0b"]),
                         ("FCb gemm", ["FCb mx cvt", "FCb gemm"])):
                i = names.index(n)
                names = names[:i] + m + names[i + 1:]
if os.environ.get("RING") == "1":  # the reference architecture on the ring chain (CVAE_KERNEL_RING)
    names = (["prologue", "C0|E0", "C1|E1", "E2", "E3", "FC", "reparam", "D0", "D1", "D2", "D3+loss", "fixup",
              "D3b", "D2b", "D1b", "D0b", "FCb", "E3b", "E2b", "E1b|C1b", "partials"])
    if os.environ.get("SUB") == "1":  # CVAE_DIAG_STAMPS=2: stamps inside the prologue, C0|E0 and FCb
        names = (["pro:issue", "pro:transform", "pro:bar", "C0+copies", "E0 gemm", "E0 epi", "C1|E1", "E2", "E3",
                  "FC", "reparam", "D0", "D1", "D2", "D3+loss", "fixup", "D3b", "D2b", "D1b", "D0b", "FCb gemm",
                  "FCb epi", "E3b", "E2b", "E1b|C1b", "partials"])
if F32:  # cvae_f32chain.h's barriers
    names = ["prologue", "C0|E0", "C1|E1", "E2", "E3", "FC", "reparam|D0 h_c", "D0 z", "D1", "D2", "D3", "loss",
             "fixup", "D3b", "D2b", "D1b", "D0b", "FCb", "E3b", "E2b", "E1b|C1b", "partials"]
for i in range(k - 1):
    print(f"{names[i]:>14s} {i:2d}: median {np.median(d[:, i]) / 1000:7.3f} us   max {d[:, i].max() / 1000:7.3f} us"
          f"   block0 {d[0, i] / 1000:7.3f} us")
ends = (st[:, k - 1] - t0) * 10 / 1000
starts = (st[:, 0] - t0) * 10 / 1000
print(f"block ends (us after the first start): block0 {ends[0]:.2f}  median {np.median(ends):.2f}  max {ends.max():.2f}"
      f" (block {int(ends.argmax())});  block0 start {starts[0]:.2f}")
# dispatch order: each block's start, in block order (8 per line: blockIdx % 8 is the XCD), and how
# much of each block's end its start explains
print("block starts (us):")
for i in range(0, nb, 8):
    print("  " + " ".join(f"{v:5.2f}" for v in starts[i:i + 8]))
dur = ends - starts
print(f"block durations: median {np.median(dur):.2f} max {dur.max():.2f} us; corr(start, end) "
      f"{np.corrcoef(starts, ends)[0, 1]:.2f}")

w = wbuf.view(NT, 8).cpu().numpy().astype(np.int64)
wid = np.nonzero(w[:, 0] > 0)[0]  # fused launch: tile blocks follow the row-chain blocks
w = w[wid]
nw = len(wid)
if len(wid) and wid[0] > 0:
    rel = lambda v: (v - t0) * 10 / 1000  # noqa: E731
    print(f"fused: chain blocks end {rel(st[:, k - 1].min()):.2f}..{rel(st[:, k - 1].max()):.2f} us after the first"
          f" chain stamp; tile work starts (pctl 0/25/50/75/100) "
          f"{[round(rel(v), 2) for v in np.percentile(w[:, 0], [0, 25, 50, 75, 100])]}"
          f", ends {[round(rel(v), 2) for v in np.percentile(w[:, 3], [0, 25, 50, 75, 100])]}")
    for lo, hi, name in ((0, 52, "group0"), (52, 168, "group1"), (168, nw, "group2")):
        g = w[lo:hi]
        print(f"  {name} tiles {lo}..{hi - 1}: start {rel(g[:, 0].min()):.2f}..{rel(g[:, 0].max()):.2f}"
              f"  end {rel(g[:, 3].min()):.2f}..{rel(g[:, 3].max()):.2f} us")
if not nw:
    sys.exit(0)
rc_end = st[:, k - 1].max()
print(f"wgrad: blocks={nw}; first entry {(w[:, 0].min() - rc_end) * 10 / 1000:.2f} us after the last row-chain stamp;"
      f" span {(w[:, 3].max() - w[:, 0].min()) * 10 / 1000:.2f} us")
print(f"  entry spread {(w[:, 0].max() - w[:, 0].min()) * 10 / 1000:.2f} us;"
      f" phases median/max us: mfma {np.median(w[:, 1] - w[:, 0]) / 100:.2f}/{(w[:, 1] - w[:, 0]).max() / 100:.2f}"
      f"  reduce {np.median(w[:, 2] - w[:, 1]) / 100:.2f}/{(w[:, 2] - w[:, 1]).max() / 100:.2f}"
      f"  adam {np.median(w[:, 3] - w[:, 2]) / 100:.2f}/{(w[:, 3] - w[:, 2]).max() / 100:.2f}")
if (w[:, 6] > 0).all():
    ph = lambda a, b: f"{np.median(w[:, b] - w[:, a]) / 100:.2f}/{(w[:, b] - w[:, a]).max() / 100:.2f}"  # noqa: E731
    print(f"  detail median/max us: first chunk {ph(0, 7)}  rest of loop {ph(7, 1)}  apply4 {ph(2, 4)}"
          f"  bias+image {ph(4, 5)}  operand stores {ph(5, 6)}  final barrier {ph(6, 3)}")
late = np.argsort(w[:, 3])[-8:]
print("  last blocks to finish (block: entry, exit us rel. first entry):",
      [(int(b), round((w[b, 0] - w[:, 0].min()) / 100, 2), round((w[b, 3] - w[:, 0].min()) / 100, 2)) for b in late])
