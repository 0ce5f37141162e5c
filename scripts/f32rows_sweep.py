"""fp32 chain row tiling vs batch (GPU box): µs per fused training step (chain + dW ⊕ Adam) of the
reference's configuration (S=10, D=3, fp32) with 4-row and 16-row chain workgroups
(CVAE_F32_ROWS), over batches 8 .. 1024 — where CVAE_F32_R4_MAX's default comes from.

  python scripts/f32rows_sweep.py > gpurun_out/<tag>/f32rows.txt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "defensive-model-vae_amd"))
import cvae_amd  # noqa: E402


def step_us(rows, B, n=200, reps=3):
    os.environ["CVAE_F32_ROWS"] = str(rows)
    torch.manual_seed(0)
    m = cvae_amd.ConditionalTrajectoryVAE(10, 3, 8)
    e = m.attach(dtype="fp32", max_batch=B, device="cuda:0", seed=1)
    del os.environ["CVAE_F32_ROWS"]
    assert e.train_kernel == "f32" and e.chain_rows(B) == rows
    x = e.as_input(torch.randn(B, 10, 3) * 3, keep_f32=True)
    e.train_steps(x, 20)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        e.train_steps(x, n)
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / n)
    e.close()
    return best


def main():
    print(f"{'B':>6} {'rows4 us':>9} {'rows16 us':>10} {'16/4':>6}")
    for B in (8, 32, 64, 96, 128, 192, 256, 512, 1024):
        t4, t16 = step_us(4, B), step_us(16, B)
        print(f"{B:6d} {t4:9.2f} {t16:10.2f} {t16 / t4:6.2f}", flush=True)


if __name__ == "__main__":
    main()
