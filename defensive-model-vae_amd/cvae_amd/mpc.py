"""MPC path tracking on the GPU: the step after generation.

Mirrors ``MPC/MPC_Tracking.py``'s interface — ``VehicleModel`` (`:23-86`), ``PathInterpolator``
(`:89-277`), ``MPCController`` (`:280-415`), ``PathTracker`` (`:418-523`) — over the HIP kernels of
``csrc/cvae_mpc.h`` (C-ABI ``cvae_mpc_track / cvae_mpc_solve / cvae_mpc_reference``).  The
reference tracks one trajectory per Python loop; ``track_batch`` tracks a whole batch of generated
trajectories in one launch (one wavefront per trajectory), which is how ``Distribution.py:114-``
uses it (every CSV's generated trajectory tracked in turn).

The MPC sub-problem is solved to its KKT point (projected Newton, exact derivatives) instead of
scipy SLSQP's finite-difference iteration with ftol 1e-6; DESIGN.md §0 (f4) states the parity
bound against the reference's own runs (tests/golden/mpc.npz).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from ._lib import CvaeMpcConfig, check, lib


def mpc_config(prediction_horizon=10, control_horizon=5, dt=0.01, wheelbase=2.8, max_steer=0.5, max_accel=7.0,
               Q=(20.0, 5.0), R=(1.0, 50.0), Qf=(20.0, 5.0), tol=1e-10, max_iter=50):
    """The C-ABI configuration; defaults = the reference's (MPC_Tracking.py:26, :283-306)."""
    if control_horizon > prediction_horizon:
        raise ValueError("control_horizon must not exceed prediction_horizon")  # :300-301
    c = CvaeMpcConfig()
    check(lib().cvae_mpc_default_config(C.byref(c)), "cvae_mpc_default_config")
    c.wheelbase, c.max_steer, c.max_accel, c.dt = float(wheelbase), float(max_steer), float(max_accel), float(dt)
    c.q_theta, c.q_v = map(float, Q)
    c.r_accel, c.r_steer = map(float, R)
    c.qf_theta, c.qf_v = map(float, Qf)
    c.tol, c.max_iter = float(tol), int(max_iter)
    c.prediction_horizon, c.control_horizon = int(prediction_horizon), int(control_horizon)
    return c


def _torch():
    import torch
    return torch


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream(torch, dev):
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _check_waypoints(wp):
    wp = np.asarray(wp, dtype=np.float64)
    if wp.ndim != 2 or wp.shape[1] != 3:
        raise ValueError("waypoints must be [n, 3] = (x, y, t)")
    if len(wp) < 2:
        raise ValueError("at least 2 waypoints are needed")  # :114-115
    if len(wp) > 64:
        raise ValueError("at most 64 waypoints per path")
    if not np.all(np.diff(wp[:, 2]) > 0):
        raise ValueError("waypoint times must be strictly increasing")  # :118-119
    if not wp[0, 2] + (wp[1, 2] - wp[0, 2]) / 2 > 0.0:
        raise ValueError("the velocity sample times [0, t[:-1] + dt/2] must increase")
    return wp


def wrap_initial_state(initial_state):
    """PathTracker.__init__ (:435-436): theta < -2.8 → theta + 2π, IN PLACE like the reference."""
    if initial_state[2] < -2.8:
        initial_state[2] = initial_state[2] + 2 * np.pi
    return initial_state


def _pack(waypoints_list, initial_states, dev):
    torch = _torch()
    wps = [_check_waypoints(w) for w in waypoints_list]
    offs = np.zeros(len(wps) + 1, np.int32)
    offs[1:] = np.cumsum([len(w) for w in wps])
    init = np.asarray(initial_states, dtype=np.float64).reshape(len(wps), 5)
    flat = np.concatenate(wps) if wps else np.zeros((0, 3))
    return (torch.from_numpy(np.ascontiguousarray(flat)).to(dev), torch.from_numpy(offs).to(dev),
            torch.from_numpy(np.ascontiguousarray(init)).to(dev))


def track_batch(waypoints_list, initial_states, total_times=None, device="cuda", return_iters=False, **cfg):
    """``PathTracker(wp, init, ...).run_simulation(total_time)`` for every path at once.

    waypoints_list: sequence of [n_p, 3] (x, y, t) arrays; initial_states: [P, 5] (x, y, theta,
    vx, vy) — theta is wrapped here as the reference's constructor does (the caller's array is
    not modified); total_times: per path (default: the path's last waypoint time, as
    ``Distribution.py:104``).  Returns a list of (times, states, controls) per path."""
    torch = _torch()
    c = mpc_config(**cfg)
    dev = torch.device(device)
    init = np.array(initial_states, dtype=np.float64).reshape(-1, 5)
    for row in init:
        wrap_initial_state(row)
    P = len(waypoints_list)
    if total_times is None:
        total_times = [float(np.asarray(w)[-1, 2]) for w in waypoints_list]
    n_steps = np.array([int(float(T) / c.dt) for T in np.broadcast_to(np.asarray(total_times, dtype=np.float64), (P,))],
                       np.int32)  # run_simulation :505
    if (n_steps < 0).any():
        raise ValueError("total_time must be >= 0")
    soff = np.zeros(P + 1, np.int64)
    soff[1:] = np.cumsum(n_steps)
    d_wp, d_off, d_init = _pack(waypoints_list, init, dev)
    d_ns = torch.from_numpy(n_steps).to(dev)
    d_so = torch.from_numpy(soff).to(dev)
    tot = int(soff[-1])
    d_states = torch.empty((tot + P, 4), dtype=torch.float64, device=dev)
    d_ctrl = torch.empty((max(tot, 1), 2), dtype=torch.float64, device=dev)
    d_it = torch.empty(max(tot, 1), dtype=torch.int32, device=dev)
    check(lib().cvae_mpc_track(C.byref(c), P, _ptr(d_wp), _ptr(d_off), _ptr(d_init), _ptr(d_ns), _ptr(d_so),
                               _ptr(d_states), _ptr(d_ctrl), _ptr(d_it), _stream(torch, dev)), "cvae_mpc_track")
    states, ctrl, its = d_states.cpu().numpy(), d_ctrl.cpu().numpy(), d_it.cpu().numpy()
    out = []
    for p in range(P):
        ns, o = int(n_steps[p]), int(soff[p])
        times = np.empty(ns + 1)
        times[0] = 0.0
        times[1:] = np.arange(ns) * c.dt + c.dt  # current_time + dt, current_time = i * dt (:491, :513)
        r = (times, states[o + p:o + p + ns + 1].copy(), ctrl[o:o + ns].copy().reshape(ns, 2))
        out.append(r + (its[o:o + ns].copy(),) if return_iters else r)
    return out


def solve_batch(states, refs, lasts, device="cuda", **cfg):
    """``MPCController.solve_mpc`` for independent sub-problems: states [n, 4] (x, y, theta, v),
    refs [n, N+1, 2] (theta_ref, v_ref), lasts [n, 2] (NaN = no previous control).
    Returns (u [n, CH, 2], cost [n], iters [n])."""
    torch = _torch()
    c = mpc_config(**cfg)
    dev = torch.device(device)
    st = torch.from_numpy(np.ascontiguousarray(states, dtype=np.float64).reshape(-1, 4)).to(dev)
    n = st.shape[0]
    ref = np.ascontiguousarray(refs, dtype=np.float64)
    if ref.shape != (n, c.prediction_horizon + 1, 2):
        raise ValueError(f"refs must be [{n}, {c.prediction_horizon + 1}, 2]")
    d_ref = torch.from_numpy(ref).to(dev)
    d_last = torch.from_numpy(np.ascontiguousarray(lasts, dtype=np.float64).reshape(n, 2)).to(dev)
    u = torch.empty((n, c.control_horizon, 2), dtype=torch.float64, device=dev)
    cost = torch.empty(n, dtype=torch.float64, device=dev)
    it = torch.empty(n, dtype=torch.int32, device=dev)
    check(lib().cvae_mpc_solve(C.byref(c), n, _ptr(st), _ptr(d_ref), _ptr(d_last), _ptr(u), _ptr(cost), _ptr(it),
                               _stream(torch, dev)), "cvae_mpc_solve")
    return u.cpu().numpy(), cost.cpu().numpy(), it.cpu().numpy()


def reference_batch(waypoints_list, initial_states, t, device="cuda"):
    """PathInterpolator queries for many paths: ([P, n_t, 5] (x, y, vx, vy, heading), [P, 6]
    (start_theta, end_vx, end_vy, end_theta, end_x, end_y))."""
    torch = _torch()
    dev = torch.device(device)
    init = np.array(initial_states, dtype=np.float64).reshape(-1, 5)
    d_wp, d_off, d_init = _pack(waypoints_list, init, dev)
    tt = np.ascontiguousarray(np.atleast_1d(np.asarray(t, dtype=np.float64)))
    d_t = torch.from_numpy(tt).to(dev)
    P = len(waypoints_list)
    out = torch.empty((P, len(tt), 5), dtype=torch.float64, device=dev)
    sc = torch.empty((P, 6), dtype=torch.float64, device=dev)
    check(lib().cvae_mpc_reference(P, _ptr(d_wp), _ptr(d_off), _ptr(d_init), _ptr(d_t), len(tt), _ptr(out), _ptr(sc),
                                   _stream(torch, dev)), "cvae_mpc_reference")
    return out.cpu().numpy(), sc.cpu().numpy()


class VehicleModel:
    """VehicleModel (:23-86): kinematic bicycle, Euler integration (host helper; the tracker's own
    rollouts run on the device)."""

    def __init__(self, wheelbase: float = 2.8, max_steer: float = 0.5, max_accel: float = 7.0):
        self.L, self.max_steer, self.max_accel = wheelbase, max_steer, max_accel

    def dynamics(self, state, control, dt):
        x, y, theta, v = state
        a = np.clip(control[0], -self.max_accel, self.max_accel)
        delta = np.clip(control[1], -self.max_steer, self.max_steer)
        return np.array([v * np.cos(theta), v * np.sin(theta), v * np.tan(delta) / self.L, a])

    def predict_trajectory(self, initial_state, controls, dt):
        states = np.zeros((len(controls) + 1, 4))
        states[0] = initial_state
        for i in range(len(controls)):
            states[i + 1] = states[i] + self.dynamics(states[i], controls[i], dt) * dt
        return states


class PathInterpolator:
    """PathInterpolator (:89-277) evaluated by the device kernel (``cvae_mpc_reference``)."""

    def __init__(self, waypoints, initial_state, device="cuda"):
        self.waypoints = _check_waypoints(waypoints)
        self.initial_state = np.asarray(initial_state, dtype=np.float64)
        self.device = device
        self.t_start, self.t_end = float(self.waypoints[0, 2]), float(self.waypoints[-1, 2])
        _, sc = reference_batch([self.waypoints], self.initial_state[None], [0.0], device)
        (self.start_theta, self.end_vx, self.end_vy, self.end_theta, self.end_x, self.end_y) = map(float, sc[0])

    def _q(self, t):
        out, _ = reference_batch([self.waypoints], self.initial_state[None], t, self.device)
        return out[0]

    def get_reference(self, t):
        x, y, vx, vy, _ = self._q(t)[0]
        return float(x), float(y), float(vx), float(vy)

    def get_reference_heading(self, t):
        return float(self._q(t)[0, 4])


class MPCController:
    """MPCController (:280-415): ``solve_mpc(current_state, reference_trajectory)`` on the device,
    keeping ``last_control`` like the reference."""

    def __init__(self, vehicle_model: VehicleModel, prediction_horizon: int = 10, control_horizon: int = 5,
                 dt: float = 0.01, device="cuda"):
        if control_horizon > prediction_horizon:
            raise ValueError("control_horizon must not exceed prediction_horizon")
        self.vehicle, self.prediction_horizon, self.control_horizon, self.dt = (vehicle_model, prediction_horizon,
                                                                                control_horizon, dt)
        self.Q, self.R, self.Qf = np.diag([20.0, 5.0]), np.diag([1.0, 50.0]), np.diag([20.0, 5.0])
        self.last_control = None
        self.device = device

    def _cfg(self):
        return dict(prediction_horizon=self.prediction_horizon, control_horizon=self.control_horizon, dt=self.dt,
                    wheelbase=self.vehicle.L, max_steer=self.vehicle.max_steer, max_accel=self.vehicle.max_accel,
                    Q=np.diag(self.Q), R=np.diag(self.R), Qf=np.diag(self.Qf))

    def solve_mpc(self, current_state, reference_trajectory):
        last = np.full(2, np.nan) if self.last_control is None else self.last_control
        u, _, _ = solve_batch(np.asarray(current_state)[None], np.asarray(reference_trajectory)[None], last[None],
                              self.device, **self._cfg())
        self.last_control = u[0, 0].copy()
        return u[0]


class PathTracker:
    """PathTracker (:418-523): ``run_simulation(total_time)`` → (times, states, controls), one
    device launch for the whole run."""

    def __init__(self, waypoints, initial_state, wheelbase: float = 2.8, prediction_horizon: int = 10,
                 control_horizon: int = 5, dt: float = 0.01, device="cuda"):
        wrap_initial_state(initial_state)
        s = np.array(initial_state, dtype=np.float64).copy()
        self.initial_state = np.array(initial_state, dtype=np.float64)
        self.waypoints = _check_waypoints(waypoints)
        self.dt = dt
        self.current_state = np.array([s[0], s[1], s[2], math.sqrt(s[3] ** 2 + s[4] ** 2)])
        self.vehicle = VehicleModel(wheelbase=wheelbase)
        self.mpc = MPCController(self.vehicle, prediction_horizon, control_horizon, dt, device)
        self.device = device
        self.trajectory = [self.current_state.copy()]
        self.controls = []
        self.times = [0.0]
        self._path_interp = None

    @property
    def path_interp(self):
        if self._path_interp is None:
            self._path_interp = PathInterpolator(self.waypoints, self.initial_state, self.device)
        return self._path_interp

    def run_simulation(self, total_time: float):
        (times, states, controls), = track_batch([self.waypoints], self.initial_state[None], [total_time],
                                                 self.device, **self.mpc._cfg())
        self.times, self.trajectory, self.controls = list(times), list(states), list(controls)
        self.current_state = states[-1].copy()
        if len(controls):
            self.mpc.last_control = controls[-1].copy()
        return times, states, controls
