"""GPU box: is the training step host-bound?  Times K eager train_step calls against the sum of
their kernel times, and the Python cost of one call (with the GPU kept busy)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "defensive-model-vae_amd")]
import torch
from cvae_amd import ConditionalTrajectoryVAE
torch.manual_seed(0)
m = ConditionalTrajectoryVAE(100, 6, 8)
eng = m.attach(dtype="bf16", max_batch=1024)
x = eng.as_input(torch.randn(1024, 100, 6))
for _ in range(50):
    eng.train_step(x)
torch.cuda.synchronize()
K = 400
eng.set_timing(True)
t0 = time.perf_counter()
for _ in range(K):
    eng.train_step(x)
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
kt = eng.kernel_times()
eng.set_timing(False)
print(f"eager: wall {t_all / K * 1e6:.1f} us/step, host enqueue {t_host / K * 1e6:.1f} us/step, kernels",
      {k: round(v[0] * 1e3, 2) for k, v in kt.items()})
t0 = time.perf_counter()
for _ in range(K):
    eng.train_step(x)
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"eager (no timing events): wall {t_all / K * 1e6:.1f} us/step, host enqueue {t_host / K * 1e6:.1f} us/step")
