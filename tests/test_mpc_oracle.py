"""SURVEY §8f-4 oracle pin: oracle/mpc_oracle.py (CPU restatement of MPC/MPC_Tracking.py on scipy)
against the reference's own runs (tests/golden/mpc.npz, tests/golden/make_mpc_goldens.py).
Bit-exact: the restatement keeps the reference's float64 operation order, so scipy's SLSQP
follows the same finite-difference iterates."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import mpc_oracle as O  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "mpc.npz")


@pytest.fixture(scope="module")
def gold():
    d = np.load(GOLD)
    return d, json.loads(bytes(d["meta"]).decode())["cases"]


def _init(d, k):
    return d[f"c{k}/init"].copy()


def test_interpolator_matches_reference(gold):
    d, cases = gold
    for k, c in enumerate(cases):
        ip = O.Interp(d[f"c{k}/waypoints"], O_wrapped(_init(d, k)))
        sc = np.array([ip.start_theta, ip.end_vx, ip.end_vy, ip.end_theta, ip.end_x, ip.end_y])
        assert np.array_equal(sc, d[f"c{k}/interp_scalars"]), c["name"]
        got = np.array([list(ip.reference(t)) + [ip.heading(t)] for t in d[f"c{k}/ref_grid"]])
        assert np.array_equal(got, d[f"c{k}/ref_vals"]), c["name"]


def O_wrapped(init):
    if init[2] < -2.8:
        init[2] += 2 * np.pi
    return init


def test_slsqp_subproblems_reproduce_reference(gold):
    d, cases = gold
    for k, c in enumerate(cases):
        n = len(d[f"c{k}/sub_x"])
        picks = [0, 1, n // 2, n - 1] if c["N"] <= 10 else [0, n // 2]
        for i in picks:
            last = d[f"c{k}/sub_last"][i]
            last = None if np.isnan(last).any() else last
            u, res = O.slsqp_solve(d[f"c{k}/sub_state"][i], d[f"c{k}/sub_ref"][i], last, c["N"], c["CH"], c["dt"])
            assert np.array_equal(res.x, d[f"c{k}/sub_x"][i]) and res.fun == d[f"c{k}/sub_fun"][i], (c["name"], i)


def test_closed_loop_replays_reference(gold):
    d, cases = gold
    k = [c["name"] for c in cases].index("main")
    c = cases[k]
    steps = 60
    t, s, u = O.track(d[f"c{k}/waypoints"], _init(d, k), c["N"], c["CH"], c["dt"], total_time=steps * c["dt"] + 1e-9)
    assert np.array_equal(s, d[f"c{k}/states"][:steps + 1]) and np.array_equal(u, d[f"c{k}/controls"][:steps])
    assert np.array_equal(t, d[f"c{k}/times"][:steps + 1])


def test_kkt_point_is_never_worse_than_slsqp(gold):
    """The checker the device solver is held to: the sub-problem's KKT point costs at most what
    SLSQP's answer costs (SLSQP stops at ftol 1e-6 with finite-difference gradients)."""
    d, cases = gold
    for k, c in enumerate(cases):
        n = len(d[f"c{k}/sub_x"])
        for i in np.linspace(0, n - 1, 3 if c["N"] <= 10 else 2).astype(int):
            last = d[f"c{k}/sub_last"][i]
            last = None if np.isnan(last).any() else last
            _, f = O.kkt_solve(d[f"c{k}/sub_state"][i], d[f"c{k}/sub_ref"][i], last, c["N"], c["CH"], c["dt"])
            assert f <= d[f"c{k}/sub_fun"][i] + 1e-9 * (1 + abs(f)), (c["name"], i, f, d[f"c{k}/sub_fun"][i])


def test_effective_box_follows_the_flat_bounds():
    b = O.effective_box(5)
    # flat [a0 d0 a1 d1 a2 | d2 a3 d3 a4 d4]: the first 5 get the accel bound, the rest the steer
    # bound, each intersected with its own kind's limit
    assert np.array_equal(b, [7.0, 0.5, 7.0, 0.5, 7.0, 0.5, 0.5, 0.5, 0.5, 0.5])
