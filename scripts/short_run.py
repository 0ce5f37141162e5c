"""Decompose bench.py's short timed region (VERDICT r02 Next #1): where the time of K steps goes
when K is small (the driver runs --steps 20 --warmup 5).

Builds the bench's cfg2 fused path exactly as bench.py does, then measures on the same process:
  * t(K) = perf_counter around run(K) + synchronize, for K in 1..400, several repetitions, and the
    host enqueue time (run(K) returning) — the intercept of t(K) = a + b·K is the fixed cost;
  * the idle synchronize() and an empty-launch round trip (the floor of any timed region);
  * t(20) after 0 / 1 / 10 / 100 ms of GPU idle (clock / power-state ramp);
  * per-launch durations of the first 20 steps after idle, from the kernels' own start/end
    timestamps (cvae_kernel_times' event pairs), against a warm 200-step pass.
Writes one JSON object to stdout.
"""
import json
import os
import statistics as st
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "defensive-model-vae_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "eager"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from cvae_amd import ConditionalTrajectoryVAE
    torch.manual_seed(0)
    model = ConditionalTrajectoryVAE(100, 6, 8, 128)
    eng = model.attach(dtype="bf16", max_batch=1024, device=dev, seed=4321)
    x = eng.as_input(torch.randn(1024, 100, 6, generator=torch.Generator().manual_seed(1234)))
    B = 1024

    if mode == "prepared":
        run = eng.prepare_steps(x, batch=B)
    elif mode == "graph":
        from cvae_amd.dist import GraphedStep
        graphs = {}

        def run(k):
            g = graphs.get(k)
            if g is None:
                g = graphs[k] = GraphedStep(eng, lambda: eng.train_steps(x, k, batch=B), n=1, warmup=0)
            g.replay()
        for k in (1, 2, 5, 10, 20, 50, 100, 200, 400):  # capture outside the timed regions
            run(k)
    else:
        def run(k):
            eng.train_steps(x, k, batch=B)

    def timed(k, idle=0.0):
        torch.cuda.synchronize(dev)
        if idle:
            time.sleep(idle)
        t0 = time.perf_counter()
        run(k)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        return (t2 - t0) * 1e6, (t1 - t0) * 1e6

    out = {"mode": mode}
    run(5)  # the driver's warm-up
    torch.cuda.synchronize(dev)
    first = timed(20)
    out["first_t20_us"] = round(first[0], 1)
    out["first_t20_enqueue_us"] = round(first[1], 1)

    # idle synchronize and the empty-launch round trip
    s = []
    for _ in range(200):
        t0 = time.perf_counter()
        torch.cuda.synchronize(dev)
        s.append((time.perf_counter() - t0) * 1e6)
    out["idle_sync_us_median"] = round(st.median(s), 2)
    y = torch.zeros(1, device=dev)
    r = []
    for _ in range(200):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        y.add_(1.0)
        torch.cuda.synchronize(dev)
        r.append((time.perf_counter() - t0) * 1e6)
    out["empty_launch_roundtrip_us_median"] = round(st.median(r), 2)

    # t(K) and the enqueue time
    ks = [1, 2, 5, 10, 20, 50, 100, 200, 400]
    rows = {}
    for rep in range(7):
        for k in ks:
            tt, te = timed(k)
            rows.setdefault(k, []).append((tt, te))
    tk = {k: round(st.median([a for a, _ in v]), 1) for k, v in rows.items()}
    te = {k: round(st.median([b for _, b in v]), 1) for k, v in rows.items()}
    out["t_K_us_median"] = tk
    out["enqueue_K_us_median"] = te
    out["us_per_step_K"] = {k: round(tk[k] / k, 2) for k in ks}
    # least-squares t = a + b K over K >= 5
    kk = [k for k in ks if k >= 5]
    mk = sum(kk) / len(kk)
    mt = sum(tk[k] for k in kk) / len(kk)
    b = sum((k - mk) * (tk[k] - mt) for k in kk) / sum((k - mk) ** 2 for k in kk)
    out["fit_fixed_us"] = round(mt - b * mk, 1)
    out["fit_us_per_step"] = round(b, 3)

    # idle before the timed region
    idl = {}
    for idle in (0.0, 0.001, 0.01, 0.1, 0.5):
        v = [timed(20, idle)[0] for _ in range(5)]
        idl[str(idle)] = round(st.median(v), 1)
    out["t20_after_idle_s"] = idl

    # per-launch durations of 20 steps right after 100 ms idle vs a warm pass
    def kernel_pass(k, idle):
        torch.cuda.synchronize(dev)
        time.sleep(idle)
        eng.set_timing(True)
        run(k)
        torch.cuda.synchronize(dev)
        kt = eng.kernel_times()
        eng.set_timing(False)
        return {n: round(v[0] * 1e3, 2) for n, v in kt.items()}
    out["kernel_us_20_after_100ms_idle"] = kernel_pass(20, 0.1)
    out["kernel_us_200_warm"] = kernel_pass(200, 0.0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
