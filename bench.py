"""bench.py — trajectories/sec of the VAE training step (BASELINE.json metric) on 1..8 MI355X.

One "step" = Training_VAE.py:345-363 on one batch: relative transform → forward →
conditional_vae_loss → backward → Adam, here the fused HIP path
(rowchain kernel + wgrad⊕Adam kernel; with N>1: rowchain → wgrad → RCCL
all-reduce of the flat gradient → Adam kernel).

Workload (BASELINE configs[1]/[2]): synthetic x ~ N(0,1) of shape (1024,100,6) per GPU,
bf16 operands (fp32 master weights/Adam/loss), latent 8, hidden 128, weights
(0.1,0.1,1,1), lr 1e-3, eps from the in-kernel Philox generator.  Data resident in
HBM before timing.  N>1: B_local=1024 per rank (weak scaling), global B = 1024·N.

Prints ONE JSON line (rank 0).  `roofline` is the dominant kernel's algorithmic
FLOP per launch ÷ its average HIP-event duration over the timed region;
`cpu_baseline` times the repo's CPU oracle (a torch-CPU restatement of the
reference step, oracle/cvae_oracle.py) on the host cores for ~10 s.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "defensive-model-vae_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK = {"bf16": 2500.0, "fp32": 157.3}  # dense TFLOP/s, MI355X_MICROARCH.md chip table


def fwd_macs(S, D, Z, H, C=2):
    """F of SURVEY §8d: forward multiply-accumulates per trajectory (4+4 layers)."""
    I = S * D
    return (C * H + H * H) + (I * H + 3 * H * H) + 2 * (2 * H * Z) + ((Z + H) * H + 2 * H * H + H * I)


def flops_per_traj(S, D, Z, H, C=2):
    F = fwd_macs(S, D, Z, H, C)
    I = S * D
    return {"total": 2 * (3 * F - C * H - I * H),
            "rowchain": 2 * F + 2 * (F - C * H - I * H),  # forward + every dX
            "wgrad": 2 * F}                                # every dW


def cpu_baseline(B, S, D, Z, H, seconds):
    from oracle.cvae_oracle import OracleCVAE, oracle_step
    threads = torch.get_num_threads()
    torch.manual_seed(0)
    model = OracleCVAE(S, D, Z, H)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    x = torch.randn(B, S, D, generator=torch.Generator().manual_seed(1234))
    times = []
    oracle_step(model, opt, x)  # warm-up
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        oracle_step(model, opt, x)
        times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(B / med, 1), "unit": "trajectories/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} steps of the oracle step (Training_VAE.py:345-363 body, torch-CPU fp32, "
                      f"B={B} S={S} D={D} Z={Z} H={H}), median {med * 1e3:.2f} ms/step"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1024, help="per-GPU batch")
    ap.add_argument("--seq-len", type=int, default=100)
    ap.add_argument("--dim", type=int, default=6)
    ap.add_argument("--latent", type=int, default=8)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="HBM bytes per launch of the dominant kernel from a rocprofv3 --pmc pass")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from cvae_amd import ConditionalTrajectoryVAE
    from cvae_amd.dist import DataParallelStep

    B, S, D, Z, H = args.batch, args.seq_len, args.dim, args.latent, args.hidden
    torch.manual_seed(0)
    model = ConditionalTrajectoryVAE(S, D, Z, H)
    eng = model.attach(dtype=args.dtype, max_batch=B, device=dev, seed=4321 + rank)
    x = torch.randn(B, S, D, generator=torch.Generator().manual_seed(1234 + rank))
    x = eng.as_input(x)  # resident in HBM, operand dtype
    dp = DataParallelStep(eng)  # N=1: fused train_step; N>1: fwd/bwd → RCCL all-reduce → Adam
    dp.broadcast_params()

    def step():
        dp.step(x, batch=B, global_batch=B * world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    eng.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    kt = eng.kernel_times()
    eng.set_timing(False)
    if world > 1:
        tt = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    assert torch.isfinite(eng.loss).all(), "non-finite loss"

    if rank == 0:
        fl = flops_per_traj(S, D, Z, H)
        per_launch = {"rowchain": fl["rowchain"] * B, "wgrad": fl["wgrad"] * B, "wgrad_adam": fl["wgrad"] * B}
        dom = max((k for k in kt if k in per_launch), key=lambda k: kt[k][0])
        avg_ms = kt[dom][0]
        achieved = per_launch[dom] / (avg_ms * 1e-3) / 1e12
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 3), "peak": PEAK[args.dtype],
                "unit": "TFLOP/s", "frac": round(achieved / PEAK[args.dtype], 6),
                "traffic": args.traffic_bytes,
                "flop_per_launch": per_launch[dom], "avg_launch_ms": round(avg_ms, 5),
                "kernels_ms": {k: round(v[0], 5) for k, v in kt.items()}}
        value = world * B * args.steps / t
        res = {"metric": "trajectories/sec per ELBO step, batch=1024 seq_len=100; 1/2/4/8 MI355X",
               "value": round(value, 1), "unit": "trajectories/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(t / args.steps * 1e3, 5), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
               "data": "synthetic x~N(0,1) (seeded), random-init weights (torch.manual_seed(0))",
               "config": {"workload": f"Training_VAE step, B_local={B} S={S} D={D} Z={Z} H={H}, "
                                      f"4+4 layers, {args.dtype} operands / fp32 master+Adam",
                          "global_batch": B * world, "seq_len": S, "state_dim": D, "latent_dim": Z,
                          "hidden_dim": H, "parallelism": f"dp{world}"},
               "roofline": roof,
               "flop_per_traj": fl["total"]}
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(B, S, D, Z, H, args.cpu_seconds)
            res["speedup_vs_cpu"] = round(value / res["cpu_baseline"]["value"], 1)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
