"""MPC tracking throughput: paths tracked per second, device vs the reference's CPU
algorithm.

Workload: Distribution.py:67-105's production call — PathTracker(prediction_horizon=30,
control_horizon=20, dt = the scene's time step) over each generated 10-point trajectory for its
last waypoint time — on the waypoints and start states of the 8 CSV cases in tests/golden/mpc.npz,
replicated with ±0.2 m waypoint jitter to P paths, one launch.  The CPU baseline runs
oracle/mpc_oracle.track (the reference's scipy SLSQP algorithm, bit-identical to it on the
fixtures) on the first case for a bounded number of steps, scaled to whole paths.

    python scripts/bench_mpc.py [--paths 1024] [--cpu-steps 12]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "defensive-model-vae_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--paths", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-steps", type=int, default=12)
    a = ap.parse_args()
    import torch
    from cvae_amd import mpc
    d = np.load(os.path.join(ROOT, "tests", "golden", "mpc.npz"))
    cases = json.loads(bytes(d["meta"]).decode())["cases"]
    ks = [k for k, c in enumerate(cases) if c["N"] == 30 and c["name"] != "test0"]
    rng = np.random.default_rng(0)
    by_dt = {}
    for i in range(a.paths):
        k = ks[i % len(ks)]
        wp = d[f"c{k}/waypoints"].copy()
        wp[1:, :2] += rng.uniform(-0.2, 0.2, (len(wp) - 1, 2))
        by_dt.setdefault(cases[k]["dt"], []).append((wp, d[f"c{k}/init"], cases[k]["T"]))
    total_steps = sum(int(T / dt) for dt, v in by_dt.items() for _, _, T in v)
    times = []
    for r in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for dt, v in by_dt.items():
            mpc.track_batch([w for w, _, _ in v], np.stack([s for _, s, _ in v]), [T for _, _, T in v],
                            prediction_horizon=30, control_horizon=20, dt=dt)
        torch.cuda.synchronize()
        if r:
            times.append(time.perf_counter() - t0)
    gpu_s = float(np.median(times))
    # CPU: the reference algorithm (scipy SLSQP), a bounded sample of one path's steps
    from oracle import mpc_oracle as O
    k = ks[0]
    c = cases[k]
    t0 = time.perf_counter()
    O.track(d[f"c{k}/waypoints"], d[f"c{k}/init"], 30, 20, c["dt"], total_time=a.cpu_steps * c["dt"] + 1e-9)
    cpu_step_s = (time.perf_counter() - t0) / a.cpu_steps
    mean_steps = total_steps / a.paths
    cpu_paths_s = 1.0 / (cpu_step_s * mean_steps)
    print(json.dumps({
        "metric": "MPC-tracked paths/s (PathTracker N=30, control horizon 20, Distribution.py config)",
        "value": round(a.paths / gpu_s, 1), "unit": "paths/s", "n_gpus": 1, "dtype": "f64",
        "paths": a.paths, "mpc_steps": total_steps, "launches": len(by_dt), "wall_s": round(gpu_s, 4),
        "mpc_steps_per_s": round(total_steps / gpu_s, 1),
        "cpu_baseline": {"value": round(cpu_paths_s, 5), "unit": "paths/s", "cores": 1, "kind": "port",
                         "sample": f"oracle.track (scipy SLSQP, the reference algorithm) {a.cpu_steps} steps of "
                                   f"{cases[k]['name']}, {cpu_step_s:.3f} s/step, scaled to {mean_steps:.0f} steps/path"},
        "data": "waypoints/start states of the reference's CSV logs (tests/golden/mpc.npz) with +-0.2 m jitter"}))


if __name__ == "__main__":
    main()
