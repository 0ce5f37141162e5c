"""bench.py — trajectories/sec of the VAE training step (BASELINE.json metric) on 1..8 MI355X.

One "step" = Training_VAE.py:345-363 on one batch: relative transform → forward →
conditional_vae_loss → backward → Adam, here the fused HIP path
(rowchain kernel + wgrad⊕Adam kernel; with N>1, or --dp at N=1: rowchain → wgrad →
RCCL all-reduce of the flat gradient → Adam kernel).

Workloads:
  cfg2 (default; BASELINE configs[1]/[2]): synthetic x ~ N(0,1) of shape (1024,100,6) per GPU,
       bf16 operands (fp32 master weights/Adam/loss), latent 8, hidden 128, weights
       (0.1,0.1,1,1), lr 1e-3, eps from the in-kernel Philox generator.  Data resident in
       HBM before timing.  N>1: B_local=1024 per rank (weak scaling), global B = 1024·N.
  cfg1 (BASELINE configs[0]): the reference's own data, StaticBlindTown05 = sce1 (38×10×3,
       from the committed fixture tests/golden/sce_fixed.npz), B=32 (--batch 38 = the
       reference's default), fp32, the reference loop: one host permutation per epoch
       (DataLoader(shuffle=True)), batches 32|6, host eps — what `python Training_VAE.py`
       runs, with the epoch's rows gathered on the device; the timed steps' permutations and eps
       are drawn on the host inside the timed region and issued through cvae_train_epochs calls of
       whole epochs (1, 2, 4 .. 32 per call), each chunk drawn while the device runs the previous one
       (the fp32 ring chain, cvae_f32chain.h, and its dW decode, cvae_f32wgrad.h).
  wide (BASELINE configs[4] shape): S=200, Z=512, 8+8 layers, bf16 (or --dtype fp8).

Prints ONE JSON line (rank 0).  `roofline` is the dominant kernel's algorithmic
FLOP per launch ÷ its average launch duration (the GEMM / MFMA roofline is the headline,
BASELINE.json north_star; the HBM ceiling rides along in `other_ceiling`);
`cpu_baseline` times the repo's CPU oracle (a torch-CPU restatement of the
reference step, oracle/cvae_oracle.py) on all host cores the process may use (capped by the
container's CPU quota): the median of >= 200 steps after 20 warm-up steps.

Timing: W warm-up steps, then the K timed steps without events (value, ms_per_step), issued
through one prepared C call on one GPU (no per-call Python before the first launch) or replayed
from a captured hipGraph on the data-parallel path; a second pass of the same K steps records
each launch's own start/end timestamps for the per-kernel durations (roofline), since events
inside the timed pass perturb it.  No step runs outside the W + K the JSON reports (graph
captures execute nothing).
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

PEAK = {"bf16": 2500.0, "fp32": 157.3, "fp8": 5000.0}  # dense TFLOP/s, MI355X_MICROARCH.md chip table
HBM_PEAK_GBS = 8000.0                      # HBM3E peak, MI355X_MICROARCH.md


def fwd_macs(S, D, Z, H, C=2, n_enc=4, n_dec=4, E=0):
    """F of SURVEY §8d: forward multiply-accumulates per trajectory (4+4 layers by default); E > 0:
    the cfg4 class embedding widens the fc and decoder-L0 inputs by E (the embedding itself is a
    gather)."""
    I = S * D
    return ((C * H + H * H) + (I * H + (n_enc - 1) * H * H) + (2 * H + E) * 2 * Z
            + ((Z + H + E) * H + (n_dec - 2) * H * H + H * I))


def flops_per_traj(S, D, Z, H, C=2, n_enc=4, n_dec=4, E=0):
    F = fwd_macs(S, D, Z, H, C, n_enc, n_dec, E)
    I = S * D
    return {"total": 2 * (3 * F - C * H - I * H),
            "rowchain": 2 * F + 2 * (F - C * H - I * H),  # forward + every dX
            "wgrad": 2 * F}                                # every dW


def bytes_per_traj(S, D, Z, H, tsize, C=2, n_enc=4, n_dec=4):
    """Algorithmic HBM bytes per trajectory: the row chain reads x and writes every
    layer input xT and pre-activation gradient gT once (unpadded); the dW kernel reads them once."""
    I = S * D
    ks = [C, H] + [I] + [H] * (n_enc - 1) + [2 * H] + [Z + H] + [H] * (n_dec - 1)
    ns = [H, H] + [H] * n_enc + [2 * Z] + [H] * (n_dec - 1) + [I]
    arena = (sum(ks) + sum(ns)) * tsize
    return {"rowchain": I * tsize + arena, "wgrad": arena}


ADAM_BYTES_PER_PARAM = 28  # p, m, v read + write (24 B) + bf16/fp32 operand copies W, Wᵀ written


def weight_stream_bytes(S, D, Z, H, dtype, C=2, n_enc=4, n_dec=4):
    """Weight-fragment bytes ONE row-chain workgroup streams per launch: every
    layer's padded forward operand Wf (e4m3 where CVAE_FP8 runs the layer in fp8: padded K % 64 ==
    0) plus the padded Wᵀ of every layer whose dX the chain computes (all but the condition and
    encoder input layers).  Every workgroup streams all of it; the chain's floor is this over the
    per-CU L2 -> CU rate."""
    r32 = lambda v: (v + 31) // 32 * 32  # noqa: E731
    I = S * D
    ks = [C, H, I] + [H] * (n_enc - 1) + [2 * H, Z + H] + [H] * (n_dec - 1)
    ns = [H, H, H] + [H] * (n_enc - 1) + [2 * Z] + [H] * (n_dec - 1) + [I]
    t = 4 if dtype == "fp32" else 2
    fwd = sum(r32(n) * r32(k) * (1 if dtype == "fp8" and r32(k) % 64 == 0 else t) for k, n in zip(ks, ns))
    bwd = sum(r32(n) * r32(k) * t for i, (k, n) in enumerate(zip(ks, ns)) if i not in (0, 2))
    return fwd + bwd


# highest per-CU weight-stream rate measured in a row-chain step (wide chain, fc backward: 512 KB
# per workgroup in 4.7-4.8 us; profiles/r02k_wide_stamps.txt) — an empirical ceiling, not a spec
CU_STREAM_MAX_GBS = 109.0


def roofline(kernel, avg_ms, flop, nbytes, dtype, traffic=None):
    """Both ceilings of one kernel.  The headline is the GEMM (MFMA) roofline whenever the kernel
    does GEMM work — BASELINE.json's north_star asks for the "achieved fraction of the GEMM
    roofline" — and the HBM ceiling otherwise (Adam); the other ceiling rides along.  Which
    ceiling would bind at peak is kept in ``peak_bound`` (neither binds the row chain: it is
    latency-bound)."""
    t = avg_ms * 1e-3
    mfma = {"achieved": flop / t / 1e12, "peak": PEAK[dtype], "unit": "TFLOP/s"}
    hbm = {"achieved": nbytes / t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    peak_bound = "hbm" if nbytes / (HBM_PEAK_GBS * 1e9) > flop / (PEAK[dtype] * 1e12) else "mfma"
    bound = "mfma" if flop > 0 else "hbm"
    head, other = (hbm, mfma) if bound == "hbm" else (mfma, hbm)
    return {"bound": bound, "peak_bound": peak_bound, "kernel": kernel, "achieved": round(head["achieved"], 3),
            "peak": head["peak"],
            "unit": head["unit"], "frac": round(head["achieved"] / head["peak"], 6),
            "traffic": traffic, "flop_per_launch": flop, "bytes_per_launch": nbytes,
            "avg_launch_ms": round(avg_ms, 5),
            "other_ceiling": {"bound": "mfma" if bound == "hbm" else "hbm",
                              "achieved": round(other["achieved"], 3), "peak": other["peak"],
                              "unit": other["unit"], "frac": round(other["achieved"] / other["peak"], 6)}}


def measured_traffic(path, kernel, batch, dtype):
    """Per-launch 2·FETCH_SIZE + WRITE_SIZE of `kernel` from a committed rocprofv3 pass, if it
    was taken on this configuration (scripts/pmc_traffic.py); else None."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("config") != {"batch": batch, "dtype": dtype}:
        return None
    k = t.get("kernels", {}).get(kernel)
    return None if k is None else k["traffic_bytes"]


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """(threads to use, affinity CPUs, cgroup CPU quota or None): every CPU this process may run on
    (all host cores), capped by the container's CPU quota when one is set — threads
    past the quota are throttled, not extra cores."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline(B, S, D, Z, H, seconds, n_enc=4, n_dec=4, data=None, min_steps=200, warmup=20):
    """The oracle step (Training_VAE.py:345-363 restated in torch-CPU) on the host cores: synthetic
    N(0,1) rows, or (data) the real dataset with the reference loop's per-epoch permutation.
    BASELINE.md's setup: all host cores, the median of >= 200 timed steps after 20 warm-up steps
    (more steps while under ``seconds``)."""
    from oracle.cvae_oracle import OracleCVAE, oracle_step
    threads, aff, quota = host_cpus()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    model = OracleCVAE(S, D, Z, H, n_enc, n_dec)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    if data is None:
        x = torch.randn(B, S, D, generator=torch.Generator().manual_seed(1234))
        batches = lambda: [x]  # noqa: E731
    else:
        n = data.shape[0]
        batches = lambda: [data[p] for p in torch.randperm(n).split(B)]  # noqa: E731
    w = 0
    while w < warmup:
        for xb in batches():
            oracle_step(model, opt, xb)
            w += 1
    rows, times = 0, []
    t_end = time.perf_counter() + seconds
    while len(times) < min_steps or time.perf_counter() < t_end:
        for xb in batches():
            t0 = time.perf_counter()
            oracle_step(model, opt, xb)
            times.append(time.perf_counter() - t0)
            rows += xb.shape[0]
    torch.set_num_threads(prev_threads)
    times.sort()
    med = times[len(times) // 2]
    rows_per_step = rows / len(times)
    what = "synthetic N(0,1)" if data is None else f"sce1 data ({data.shape[0]} rows, shuffled batches)"
    return {"value": round(rows_per_step / med, 1), "unit": "trajectories/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "sample": f"median of {len(times)} steps after {w} warm-up steps of the oracle step "
                      f"(Training_VAE.py:345-363 body, torch-CPU fp32, B={B} S={S} D={D} Z={Z} H={H}, "
                      f"{n_enc}+{n_dec} layers, {what}), {med * 1e3:.3f} ms/step median, "
                      f"{sum(times) / len(times) * 1e3:.3f} mean, {threads} threads"}


def launch_plan(gpus, env, device_count):
    """What ``bench.py --gpus N`` does with the process it runs in (decided before any GPU call:
    ``torch.cuda.device_count()`` does not initialise the GPU on this image).

    Returns ("run", world) to measure in this process, ("spawn", N) to start N rank processes as
    children of this one (``--gpus N`` without a launcher), or ("error", message).
    - Under a launcher (``WORLD_SIZE`` set, e.g. ``torch.distributed.run --nproc-per-node N``) the
      launcher's world is the world; ``--gpus`` must agree with it when given.
    - Without one, N > 1 spawns N ranks (one per GPU), which needs N visible GPUs unless the ranks
      rehearse on one GPU (``CVAE_BENCH_SHARE_GPU=1``)."""
    share = env.get("CVAE_BENCH_SHARE_GPU") == "1"
    if "WORLD_SIZE" in env:
        try:
            world = int(env["WORLD_SIZE"])
        except ValueError:
            return "error", f"WORLD_SIZE={env['WORLD_SIZE']!r} is not an integer"
        if gpus is not None and gpus != world:
            return "error", (f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks: the line would "
                             f"report n_gpus={world}; run with --gpus {world}, or without a launcher")
        return "run", world
    n = 1 if gpus is None else gpus
    if n < 1:
        return "error", f"--gpus {n}: need at least one GPU"
    if n > 1 and not share and device_count < n:
        return "error", (f"--gpus {n} but only {device_count} GPU(s) are visible (CVAE_BENCH_SHARE_GPU=1 runs the "
                         f"ranks on GPU 0 as a rehearsal, not a scaling measurement)")
    return ("spawn", n) if n > 1 else ("run", 1)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n, env, port):
    """The environment of each of the n rank processes: torch.distributed.run's variables for one
    node (rendezvous on 127.0.0.1), everything else inherited (HSA_ENABLE_IPC_MODE_LEGACY=0 too).
    Ranks sharing one GPU (CVAE_BENCH_SHARE_GPU=1, a rehearsal) get one HIP hardware queue each
    (GPU_MAX_HW_QUEUES=1, whatever the environment says): with HIP's default 4 per process, 8
    processes oversubscribe the GPU's queue slots, the scheduler time-slices them, and every
    exchange wait becomes milliseconds (46 ms per step at 8 ranks against 0.18 ms with one queue
    each, profiles/r05w/)."""
    out = []
    share = env.get("CVAE_BENCH_SHARE_GPU") == "1"
    for r in range(n):
        e = dict(env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        if share:
            e["GPU_MAX_HW_QUEUES"] = "1"
        out.append(e)
    return out


def run_ranks(cmd, envs, out, grace_s=60.0, poll_s=0.05, done_grace_s=300.0):
    """Start one child per environment running ``cmd``, forward rank 0's result line to ``out``, and
    return the worst exit status (the first non-zero one in rank order among the ranks that ended by
    themselves, else 0).  Rank 0's stdout is
    read through a pipe (its other output and every other rank's stdout go to this process's
    stderr); the line forwarded is the last one that parses as a JSON object with a "metric" key.
    When a rank fails, the others get ``grace_s`` to finish (they may be blocked in a collective
    with it) and are then killed — by their own PIDs."""
    import subprocess
    import threading
    procs, lines = [], []
    for r, e in enumerate(envs):
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))

    def pump():
        for raw in procs[0].stdout:
            s = raw.decode(errors="replace").rstrip("\n")
            try:
                d = json.loads(s)
            except ValueError:
                d = None
            if isinstance(d, dict) and "metric" in d:
                lines.append(s)
            else:
                print(s, file=sys.stderr, flush=True)
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    deadline, fail_at, killed = None, None, set()
    while None in [p.poll() for p in procs]:  # a list: every child polled each round
        # a rank that failed: the rest get grace_s; one that finished cleanly while others still run
        # (rank 0's CPU-baseline leg, or a peer stuck in a collective the finished rank never entered):
        # done_grace_s, then the rest are killed
        now = time.monotonic()
        if fail_at is None and any(p.returncode not in (None, 0) for p in procs):
            fail_at = now
            deadline = min(deadline or float("inf"), now + grace_s)
        if deadline is None and any(p.returncode == 0 for p in procs):
            deadline = now + done_grace_s
        if deadline is not None and time.monotonic() > deadline:
            for r, p in enumerate(procs):
                if p.poll() is None:
                    p.kill()
                    killed.add(r)
        time.sleep(poll_s)
    th.join()
    codes = [p.wait() for p in procs]
    if lines:
        print(lines[-1], file=out, flush=True)
    # the ranks that failed by themselves first; the ones killed here only if nothing else failed
    bad = [c for r, c in enumerate(codes) if c != 0 and r not in killed] or [c for c in codes if c != 0]
    if not bad:
        return 0
    return bad[0] if bad[0] > 0 else 128 - bad[0]  # killed by signal s: the shell's 128 + s


def spawn_main(n, argv):
    """``bench.py --gpus N`` without a launcher: N rank processes, this one a plain parent that never
    touches the GPU (no exec — the ranks are children).  The ranks run this same script with the
    same arguments under torch.distributed.run's environment."""
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + list(argv)
    envs = rank_envs(n, os.environ, int(os.environ.get("MASTER_PORT") or _free_port()))
    print(f"bench.py: starting {n} rank processes (master 127.0.0.1:{envs[0]['MASTER_PORT']})", file=sys.stderr,
          flush=True)
    return run_ranks(cmd, envs, sys.stdout)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each); without a launcher N > 1 starts the N ranks as child processes; "
                         "under torch.distributed.run it must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (cfg2/wide: 1024, cfg1: 32)")
    ap.add_argument("--workload", default="cfg2", choices=["cfg2", "cfg1", "wide", "cfg4"],
                    help="cfg2: the headline (S=100, Z=8, 4+4 layers, synthetic); cfg1: the reference's sce1 "
                         "data at B=32, fp32; wide: BASELINE cfg5's shape (S=200, Z=512, 8+8 layers); cfg4: cfg2's "
                         "shape with the scenario-class embedding (4 classes, class_dim 16; a build-side extension)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32", "fp8"],
                    help="operand dtype (default: bf16; cfg1: fp32)")
    ap.add_argument("--dp", action="store_true",
                    help="data-parallel split step even at N=1: fwd/bwd → RCCL all-reduce → Adam")
    ap.add_argument("--exchange", default="auto", choices=["auto", "peer", "rccl"],
                    help="N>1 gradient exchange: peer = dW + reduce-scatter + Adam + all-gather inside the "
                         "weight-gradient launch over IPC-mapped peer memory (cvae_amd.peer); rccl = all-reduce of "
                         "the flat gradient, then Adam; auto = peer where the configuration has it")
    ap.add_argument("--torch-allreduce", action="store_true",
                    help="split step: torch.distributed's all_reduce instead of the library's own RCCL "
                         "communicator on the step's stream (cvae_rccl_*; A/B)")
    ap.add_argument("--shard-adam", action="store_true",
                    help="split step (rccl): reduce-scatter of the gradient, Adam on this rank's 1/N of the flat "
                         "state, all-gather of the parameters, repack (instead of all-reduce + the whole Adam)")
    ap.add_argument("--buckets", type=int, default=1, choices=[1, 2],
                    help="split step: 2 = decoder-gradient all-reduce overlapped with the rest of dW")
    ap.add_argument("--graph", action="store_true",
                    help="capture the step into a hipGraph and replay it (device step counters); the default "
                         "for the split (data-parallel) step")
    ap.add_argument("--no-graph", action="store_true", help="split step issued eagerly (no hipGraph)")
    ap.add_argument("--graph-steps", type=int, default=8,
                    help="training steps captured per graph replay (a remainder runs a 1-step graph)")
    ap.add_argument("--cpu-seconds", type=float, default=5.0,
                    help="CPU baseline: time at least this long (and at least 200 steps)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-b2b", action="store_true",
                    help="skip the back-to-back single-kernel pass (profiling runs: rocprof then sees step launches only)")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM traffic from rocprofv3 --pmc passes (scripts/pmc_traffic.py)")
    args = ap.parse_args()
    what, arg = launch_plan(args.gpus, os.environ, torch.cuda.device_count())
    if what == "error":
        print(f"bench.py: {arg}", file=sys.stderr, flush=True)
        sys.exit(2)
    if what == "spawn":
        sys.exit(spawn_main(arg, sys.argv[1:]))
    # ONE JSON line on stdout: native libraries (RCCL's version banner) write to fd 1 directly, so
    # fd 1 becomes stderr for the whole run and the result goes to a duplicate of the original stdout
    out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    world = arg
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N>1 path on a one-GPU box: every rank on GPU 0, gloo for the host-side
    # collectives (RCCL refuses two ranks on one GPU); the numbers are not a scaling measurement
    share = os.environ.get("CVAE_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    if world > 1 or args.dp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from cvae_amd import ConditionalTrajectoryVAE
    from cvae_amd.dist import DataParallelStep, GraphedStep

    wl = args.workload
    S, D, Z, H, NE, ND = 100, 6, 8, 128, 4, 4
    if wl == "wide":
        S, Z, NE, ND = 200, 512, 8, 8
    if wl == "cfg1":
        S, D = 10, 3
    dtype = args.dtype or ("fp32" if wl == "cfg1" else "bf16")
    B = args.batch or (32 if wl == "cfg1" else 1024)
    NC, CE = (4, 16) if wl == "cfg4" else (0, 0)  # cfg4: scenes (Town04/Town05 sce1-4) and embedding width
    torch.manual_seed(0)
    model = ConditionalTrajectoryVAE(S, D, Z, H, NE, ND, n_classes=NC, class_dim=CE or 16)
    eng = model.attach(dtype=dtype, max_batch=B, device=dev, seed=4321)
    dp = DataParallelStep(eng, force_split=args.dp, buckets=args.buckets,
                          exchange="rccl" if wl in ("cfg1", "cfg4") or args.shard_adam else args.exchange,
                          native=False if args.torch_allreduce else None, shard_adam=args.shard_adam)
    dp.broadcast_params()

    if wl == "cfg1":
        import numpy as np
        sce1 = np.load(os.path.join(ROOT, "tests", "golden", "sce_fixed.npz"))["sce1_x"]
        data_cpu = torch.from_numpy(np.ascontiguousarray(sce1, dtype=np.float32))
        n_rows = data_cpu.shape[0]
        eng.keep_f32 = True
        x = eng.as_input(data_cpu, keep_f32=True)
        idx_dev = torch.empty(n_rows, device=dev, dtype=torch.int64)
        sizes = [min(B, n_rows - s) for s in range(0, n_rows, B)]
        gen = torch.Generator().manual_seed(0)
        state = {"k": len(sizes)}
        if not dp.split and torch.cuda.is_available():
            # the engine uploads each chunk's permutations and eps through pinned staging blocks:
            # allocate one of every size class the timed chunks use now (setup), not inside the
            # timed region (a first pinned allocation costs ~0.1 ms)
            for E in range(1, 33):
                for shape, dt in (((E, n_rows), torch.int64), ((E * n_rows, Z), torch.float32)):
                    torch.empty(shape, dtype=dt).pin_memory()

        def run(k):
            """k batches of the reference loop: a fresh permutation each epoch (host, DataLoader
            shuffle) and host eps per batch (randn_like on the CPU, :205).  One GPU: the k steps'
            epochs drawn on the host and issued through cvae_train_epochs calls of whole epochs
            (what cvae_amd.train does); data-parallel: per step."""
            if not dp.split:
                # in chunks of whole epochs (the last may be cut short), as cvae_amd.train issues them:
                # a chunk's draws run on the host while the device runs the previous chunk (the engine
                # uploads through pinned memory, queued behind the kernels); chunks of 1, 2, 4 .. 32
                # epochs keep the first, unhidden draw short and every later one behind the device
                spe, left, ce = len(sizes), k, 1
                while left > 0:
                    ks = min(left, ce * spe)
                    E = (ks + spe - 1) // spe
                    perms = torch.stack([torch.randperm(n_rows, generator=gen) for _ in range(E)])
                    eps = torch.randn(E * n_rows, Z, generator=gen)
                    eng.train_epochs(x, perms, B, n_steps=ks, eps=eps)
                    left -= ks
                    ce = min(2 * ce, 32)  # each chunk's draws (~8 us an epoch) hide behind the last one's steps
                return
            for _ in range(k):
                if state["k"] == len(sizes):
                    idx_dev.copy_(torch.randperm(n_rows, generator=gen), non_blocking=True)
                    state["k"] = 0
                j = state["k"]
                lo = sum(sizes[:j])
                eps = torch.randn(sizes[j], Z, generator=gen)
                dp.step(x, idx=idx_dev[lo:lo + sizes[j]], eps=eps, batch=sizes[j],
                        global_batch=sizes[j] * world)
                state["k"] += 1
        rows_per_step = n_rows / len(sizes)
    else:
        x = torch.randn(B, S, D, generator=torch.Generator().manual_seed(1234 + rank))
        x = eng.as_input(x)  # resident in HBM, operand dtype
        cls = None
        if NC:  # cfg4: a scene class per trajectory, uniform over the NC scenes (seeded)
            cls = torch.randint(0, NC, (B,), generator=torch.Generator().manual_seed(99 + rank),
                                dtype=torch.int32).to(dev)
        ckw = {"classes": cls} if cls is not None else {}
        rows_per_step = B
        graphed = prepared = None
        use_graph = args.graph or (dp.split and dp.px is None and not args.no_graph)
        graph_note = ""
        graphed1 = None
        if dp.px is not None and not use_graph:
            # peer exchange: two launches per step, no collective call, no host work per step
            prepared = dp.px.prepare(x, B)
        elif not dp.split and not use_graph:
            # the fused steps through one prepared C call (arguments converted once): train_steps'
            # ~40 us of Python before the first launch would otherwise be a fixed cost of every
            # timed region — 1.5 us per step at the driver's 20 steps (short runs)
            prepared = eng.prepare_steps(x, batch=B, classes=cls)
        if use_graph:
            one = lambda: dp.step(x, batch=B, global_batch=B * world, **ckw)  # noqa: E731
            try:
                if dist.is_initialized():  # RCCL's communicator is created outside the capture
                    dist.all_reduce(torch.zeros(1, device=dev))
                    torch.cuda.synchronize(dev)
                # the capture executes nothing: no training step runs outside warm-up + timed steps
                graphed = GraphedStep(eng, one, n=max(1, args.graph_steps), warmup=0)
                graphed1 = graphed if graphed.n == 1 else GraphedStep(eng, one, n=1, warmup=0)
            except Exception as e:  # capture refused (e.g. a collective backend that cannot be captured)
                graphed, graph_note = None, f" (graph capture failed, eager: {type(e).__name__})"
                torch.cuda.synchronize(dev)

        def run(k):
            """k training steps: on one GPU one cvae_train_steps call (no host work per step); split
            (data-parallel) path: fwd/bwd → RCCL all-reduce → Adam per step; --graph: replays."""
            if graphed is not None:
                for _ in range(k // graphed.n):
                    graphed.replay()
                for _ in range(k % graphed.n):
                    graphed1.replay()
            elif prepared is not None:
                prepared(k)
            elif not dp.split:
                eng.train_steps(x, k, batch=B, **ckw)
            else:
                for _ in range(k):
                    dp.step(x, batch=B, global_batch=B * world, **ckw)

    run(args.warmup)
    torch.cuda.synchronize(dev)
    verified = None
    if dp.px is not None:  # the exchange's results checked once, before anything is timed
        verified = dp.verify_exchange()
        if verified is not True:
            prepared = None  # run() now steps through the RCCL all-reduce
            run(args.warmup)
            torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    verified_after = None
    if dp.px is not None:
        # the exchange checked again over the state the timed steps left (collective; every rank's
        # fault word, every rank's operand-copy checksum against the others' and against the repack
        # from the gathered master state): a failure invalidates the number
        verified_after = dp.verify_exchange(fallback=False)
        if verified_after is not True:  # no number: the line says why, the exit status says so too
            if rank == 0:
                print(json.dumps({"metric": "trajectories/sec per ELBO step, batch=1024 seq_len=100; 1/2/4/8 MI355X",
                                  "value": None, "unit": "trajectories/s", "n_gpus": world, "steps": args.steps,
                                  "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
                                  "exchange_verified": verified, "exchange_verified_after": verified_after,
                                  "invalid": f"the peer exchange failed its check after the timed steps: "
                                             f"{verified_after}"}), file=out, flush=True)
            dp.close()
            dist.destroy_process_group()
            sys.exit(3)
    elif eng.fault():  # a bounded in-kernel wait gave up inside the timed steps: no valid number
        raise RuntimeError(f"rank {rank}: fault word {eng.fault():#x} set during the timed steps "
                           f"({dp.exchange} exchange); the measurement is invalid")
    # kernel durations for the roofline: the same K steps again with HIP events recorded on the
    # launch stream between kernels (events inside the timed pass would add ~10 us per step;
    # graph replays record none, so this pass runs eagerly)
    eng.set_timing(True)
    if wl != "cfg1" and graphed is not None:
        for _ in range(args.steps):
            dp.step(x, batch=B, global_batch=B * world, **ckw)
    else:
        run(args.steps)
    torch.cuda.synchronize(dev)
    kt = eng.kernel_times()
    eng.set_timing(False)
    # each kernel alone, launched back-to-back (cvae_bench_kernels): the step's kernels without
    # their neighbours' cache/instruction-cache effects
    b2b = None
    if not args.no_b2b and wl not in ("cfg1", "cfg4") and world == 1:
        b2b = eng.bench_kernels(x, max(args.steps, 20), batch=B)
    if world > 1:
        tt = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    if not os.environ.get("CVAE_LIB"):  # diagnostic builds (scripts/bench_variants.sh) compute garbage
        assert torch.isfinite(eng.loss).all(), "non-finite loss"

    px_stats = dp.px.stats() if dp.px is not None else None
    if rank == 0:
        fl = flops_per_traj(S, D, Z, H, n_enc=NE, n_dec=ND, E=CE)
        tsize = 4 if dtype == "fp32" else 2  # fp8: bf16 activations
        bt = bytes_per_traj(S, D, Z, H, tsize, n_enc=NE, n_dec=ND)
        n_par = eng.n_params
        rows_launch = rows_per_step if wl == "cfg1" else B
        flop = {k: fl["rowchain" if k.startswith("rowchain") else "wgrad"] * rows_launch
                for k in ("rowchain", "wgrad", "wgrad_adam", "wgrad_dec", "wgrad_rest")}
        nbytes = {"rowchain": bt["rowchain"] * rows_launch, "wgrad": bt["wgrad"] * rows_launch + 4 * n_par,
                  "wgrad_adam": bt["wgrad"] * rows_launch + ADAM_BYTES_PER_PARAM * n_par,
                  "wgrad_dec": bt["wgrad"] * rows_launch, "wgrad_rest": bt["wgrad"] * rows_launch}
        flop["fused_step"] = flop["rowchain"] + flop["wgrad_adam"]
        nbytes["fused_step"] = nbytes["rowchain"] + nbytes["wgrad_adam"]
        flop["adam"], nbytes["adam"] = 0, ADAM_BYTES_PER_PARAM * n_par
        # peer exchange: every dW tile over the local rows + Adam on this rank's 1/world of the tiles
        flop["px_wgrad"] = flop["wgrad"]
        nbytes["px_wgrad"] = bt["wgrad"] * rows_launch + ADAM_BYTES_PER_PARAM * n_par // max(world, 1)
        dom = max((k for k in kt if k in flop and flop[k] > 0), key=lambda k: kt[k][0])
        std = (S, D, Z, H, NE, ND) == (100, 6, 8, 128, 4, 4)
        # BASELINE cfg5's shape: its own committed pass (gpu_round.sh, profiles/traffic_wide_<dtype>.json)
        tfile = args.traffic_file if std else (os.path.join(ROOT, "profiles", f"traffic_wide_{dtype}.json")
                                              if (S, D, Z, H, NE, ND) == (200, 6, 512, 128, 8, 8) else None)
        traffic = measured_traffic(tfile, dom, B, dtype) if tfile else None
        roof = roofline(dom, kt[dom][0], flop[dom], nbytes[dom], dtype, traffic)
        if "rowchain" in kt and wl != "cfg1":
            wsb = weight_stream_bytes(S, D, Z, H, dtype, n_enc=NE, n_dec=ND)
            ach = wsb / (kt["rowchain"][0] * 1e-3) / 1e9
            roof["weight_stream"] = {"kernel": "rowchain", "bytes_per_workgroup": wsb,
                                     "achieved_GBps_per_CU": round(ach, 1),
                                     "measured_max_GBps_per_CU": CU_STREAM_MAX_GBS,
                                     "frac": round(ach / CU_STREAM_MAX_GBS, 4),
                                     "active_CUs": (rows_launch + 15) // 16}
        roof["kernels_ms"] = {k: round(v[0], 5) for k, v in kt.items()}
        if b2b:
            roof["kernels_back_to_back_ms"] = {k: round(v, 5) for k, v in b2b.items()}
        value = world * rows_per_step * args.steps / t
        if wl == "cfg2":
            metric = "trajectories/sec per ELBO step, batch=1024 seq_len=100; 1/2/4/8 MI355X"
            data = "synthetic x~N(0,1) (seeded), random-init weights (torch.manual_seed(0))"
        elif wl == "cfg1":
            metric = (f"trajectories/sec per ELBO step, sce1 StaticBlindTown05 data, batch={B} seq_len=10 "
                      f"(BASELINE configs[0])")
            data = "the reference's trajectory_sce1_cond.npy rows (38x10x3, committed fixture), host eps"
        elif wl == "cfg4":
            metric = (f"trajectories/sec per ELBO step, batch={B} seq_len={S}, scenario-class embedding "
                      f"(BASELINE configs[3])")
            data = (f"synthetic x~N(0,1) and class ids uniform over {NC} scenes (seeded), random-init weights "
                    f"(torch.manual_seed(0)); class_dim {CE}; parity unpinned vs the reference (no such model)")
        else:
            metric = f"trajectories/sec per ELBO step, batch={B} seq_len={S} (BASELINE cfg5 shape)"
            data = "synthetic x~N(0,1) (seeded), random-init weights (torch.manual_seed(0))"
        if wl == "cfg1":
            path = "split" if dp.split else "fused"
        elif dp.px is not None:
            path = "peer-exchange (dW + reduce-scatter + Adam + all-gather in one launch, no collective)"
        else:
            path = (("graphed " if graphed is not None else "") + ("split" if dp.split else "fused")
                    + (f" x{graphed.n}/replay" if graphed is not None and graphed.n > 1 else "") + graph_note)
        res = {"metric": metric,
               "value": round(value, 1), "unit": "trajectories/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(t / args.steps * 1e3, 5), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": data,
               "config": {"workload": f"{wl}: Training_VAE step, B_local={B} S={S} D={D} Z={Z} H={H}, "
                                      f"{NE}+{ND} layers, {dtype} operands / fp32 master+Adam, {path} step"
                                      + ((", sharded Adam (reduce-scatter, Adam on 1/N, all-gather, repack)" if dp.shard_adam else
                                          f", rccl all-reduce ({'library communicator on the step stream' if dp.rccl is not None else 'torch.distributed'}), {args.buckets} buckets")
                                         if dp.split and dp.px is None else "") + (f" [{dp.exchange_note}]" if dp.exchange_note else ""),
                          "global_batch": B * world, "seq_len": S, "state_dim": D, "latent_dim": Z,
                          "hidden_dim": H, "parallelism": f"dp{world}" + (" (rehearsal: all ranks on GPU 0)"
                                                                          if share else "")},
               "roofline": roof,
               "flop_per_traj": fl["total"]}
        if px_stats is not None:
            res["exchange_waits_rank0"] = px_stats
            k_gpu, g_blocks = dp.px.layout()
            res["exchange_layout"] = {"ranks_on_gpu": k_gpu, "tile_blocks": g_blocks,
                                      "operand_checksum": f"{dp.px.last_checksum:#018x}"}
        if verified is not None:  # the peer exchange's warm-up self-check (PeerExchange.verify)
            res["exchange_verified"] = verified
        if verified_after is not None:  # the same check after the timed steps (a failure exits above)
            res["exchange_verified_after"] = verified_after
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(B, S, D, Z, H, args.cpu_seconds, NE, ND,
                                               data=data_cpu if wl == "cfg1" else None)
            res["speedup_vs_cpu"] = round(value / res["cpu_baseline"]["value"], 1)
        print(json.dumps(res), file=out, flush=True)
    dp.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
