"""CPU oracle for the MPC path tracker — TEST INFRASTRUCTURE.

Only ``tests/`` may import this module; the product path (``cvae_amd.mpc``) runs the HIP kernels
of ``csrc/cvae_mpc.h`` and has no host fallback.

A restatement of ``MPC/MPC_Tracking.py`` on its own third-party dependency, scipy (1.15.3 here):
``scipy.interpolate.interp1d`` for the path splines and ``scipy.optimize.minimize(method='SLSQP')``
for the sub-problem, each function citing the reference lines it follows.  The objective keeps
the reference's operation order (a Python loop over the horizon), so SLSQP's finite-difference
iterates are reproduced; ``tests/test_mpc_oracle.py`` pins this module to the reference's own runs
(tests/golden/mpc.npz, made by tests/golden/make_mpc_goldens.py).

``kkt_solve`` is the independent checker for the device solver: the same sub-problem solved to
high accuracy with analytic gradients (L-BFGS-B on the effective box).
"""
from __future__ import annotations

import numpy as np
from scipy.interpolate import interp1d
from scipy.optimize import minimize

DEG = np.pi / 180


def _wrap(th):
    return th if th >= -2.8 else th + 2 * np.pi  # :202, :211, :273


def _kind(n):
    return "cubic" if n >= 4 else "quadratic" if n >= 3 else "linear"  # :125-137, :172-178


class Interp:
    """PathInterpolator (:89-277)."""

    def __init__(self, wp, init):
        t, x, y = wp[:, 2], wp[:, 0], wp[:, 1]
        self.t_start, self.t_end = float(t[0]), float(t[-1])
        f = lambda tt, v, k: interp1d(tt, v, kind=k, bounds_error=False, fill_value="extrapolate")  # noqa: E731
        self.fx, self.fy = f(t, x, _kind(len(t))), f(t, y, _kind(len(t)))
        dt = np.diff(t)
        dt = np.where(dt == 0, 1e-6, dt)
        vx = np.concatenate(([init[-2]], np.diff(self.fx(t)) / dt))  # :145-163
        vy = np.concatenate(([init[-1]], np.diff(self.fy(t)) / dt))
        tv = np.concatenate(([0.0], t[:-1] + dt / 2))
        self.fvx, self.fvy = f(tv, vx, _kind(len(tv))), f(tv, vy, _kind(len(tv)))
        self.end_x, self.end_y = float(self.fx(self.t_end)), float(self.fy(self.t_end))  # :194-195
        self.start_theta = _wrap(float(np.arctan2(float(self.fvy(self.t_start)), float(self.fvx(self.t_start)))))
        self.end_vx = self.end_vy = None
        for t1 in np.arange(0, t[-1] + 0.001, 0.001):  # :204-218
            th = _wrap(float(np.arctan2(float(self.fvy(t1)), float(self.fvx(t1)))))
            if abs(th - self.start_theta) > 45 * np.pi / 180:
                tm = (t[-1] + t[-2]) / 2
                self.end_vx, self.end_vy = float(self.fvx(tm)), float(self.fvy(tm))
                break
        if self.end_vx is None:
            self.end_vx, self.end_vy = float(self.fvx(self.t_end)), float(self.fvy(self.t_end))
        self.end_theta = _wrap(float(np.arctan2(self.end_vy, self.end_vx)))

    def reference(self, t):
        """get_reference (:224-252)."""
        if t <= self.t_end:
            x, y = float(self.fx(t)), float(self.fy(t))
            vx, vy = float(self.fvx(t)), float(self.fvy(t))
            if abs(float(np.arctan2(vy, vx)) - self.start_theta) > 90 * np.pi / 180:
                vx, vy = self.end_vx, self.end_vy
            return x, y, vx, vy
        de = t - self.t_end
        return self.end_x + self.end_vx * de, self.end_y + self.end_vy * de, self.end_vx, self.end_vy

    def heading(self, t):
        """get_reference_heading (:254-277)."""
        th = self.end_theta if t > self.t_end else np.arctan2(*self.reference(t)[2:4][::-1])
        return _wrap(th)


def dynamics(state, control, L=2.8, max_steer=0.5, max_accel=7.0):
    """VehicleModel.dynamics (:39-64)."""
    x, y, theta, v = state
    a = np.clip(control[0], -max_accel, max_accel)
    d = np.clip(control[1], -max_steer, max_steer)
    return np.array([v * np.cos(theta), v * np.sin(theta), v * np.tan(d) / L, a])


def objective(u_flat, state, ref, last, N, CH, dt, L=2.8, Q=(20.0, 5.0), R=(1.0, 50.0), Qf=(20.0, 5.0)):
    """solve_mpc's objective (:329-373), in the reference's operation order."""
    Qm, Rm, Qfm = np.diag(Q), np.diag(R), np.diag(Qf)
    u = u_flat.reshape(CH, 2)
    full = np.zeros((N, 2))
    full[:CH] = u
    if CH < N:
        full[CH:] = u[-1]
    st = np.zeros((N + 1, 4))
    st[0] = state
    for i in range(N):  # predict_trajectory (:66-86)
        st[i + 1] = st[i] + dynamics(st[i], full[i], L) * dt
    cost = 0.0
    for i in range(N + 1):
        e = st[i, 2:4] - ref[i]
        cost += e.T @ (Qm if i < N else Qfm) @ e
    for i in range(CH):
        if i == 0:
            du = np.zeros(2) if last is None else u[0] - last
        else:
            du = u[i] - u[i - 1]
        cost += du.T @ Rm @ du
    return cost


def slsqp_solve(state, ref, last, N, CH, dt, L=2.8, max_steer=0.5, max_accel=7.0):
    """solve_mpc (:311-415) with scipy SLSQP; returns (control sequence [CH, 2], result)."""
    u0 = np.zeros((CH, 2))
    if last is not None:
        u0[0] = last.copy()

    def cons(uf):
        u = uf.reshape(CH, 2)
        return np.array([c for i in range(CH) for c in (max_accel - u[i, 0], u[i, 0] + max_accel,
                                                         max_steer - u[i, 1], u[i, 1] + max_steer)])

    bounds = [(-max_accel, max_accel)] * CH + [(-max_steer, max_steer)] * CH  # over the FLAT vector (:390-394)
    res = minimize(objective, u0.flatten(), args=(state, ref, last, N, CH, dt, L), method="SLSQP", bounds=bounds,
                   constraints={"type": "ineq", "fun": cons}, options={"maxiter": 100, "ftol": 1e-6})
    if res.success:
        return res.x.reshape(CH, 2), res
    return u0, res


def effective_box(CH, max_steer=0.5, max_accel=7.0):
    """Per flat index: the SLSQP bound intersected with the constraint of the variable's kind."""
    b = np.array([max_accel if f < CH else max_steer for f in range(2 * CH)])
    kind = np.array([max_accel if f % 2 == 0 else max_steer for f in range(2 * CH)])
    return np.minimum(b, kind)


def _grad(u_flat, state, ref, last, N, CH, dt, L, Q, R, Qf):
    """Analytic gradient of ``objective`` (forward rollout + adjoint)."""
    u = u_flat.reshape(CH, 2)
    c = np.minimum(np.arange(N), CH - 1)
    a, d = u[c, 0], u[c, 1]
    v = np.empty(N + 1)
    th = np.empty(N + 1)
    v[0], th[0] = state[3], state[2]
    for i in range(N):
        th[i + 1] = th[i] + v[i] * np.tan(d[i]) / L * dt
        v[i + 1] = v[i] + a[i] * dt
    q = np.array([Q] * N + [Qf])
    eth, ev = th - ref[:, 0], v - ref[:, 1]
    lam_th = 2 * q[:, 0] * eth  # dJ/dtheta_k
    lam_v = 2 * q[:, 1] * ev
    g = np.zeros((CH, 2))
    # backward pass: adjoints of theta and v
    at, av = lam_th[N], lam_v[N]
    for i in range(N - 1, -1, -1):
        g[c[i], 0] += av * dt
        g[c[i], 1] += at * v[i] / L * dt / np.cos(d[i]) ** 2
        av = lam_v[i] + av + at * np.tan(d[i]) / L * dt
        at = lam_th[i] + at
    Rv = np.array(R)
    for i in range(CH):
        prev = (None if last is None else last) if i == 0 else u[i - 1]
        if prev is not None:
            g[i] += 2 * Rv * (u[i] - prev)
        if i + 1 < CH:
            g[i] -= 2 * Rv * (u[i + 1] - u[i])
    return g.ravel()


def kkt_solve(state, ref, last, N, CH, dt, L=2.8, Q=(20.0, 5.0), R=(1.0, 50.0), Qf=(20.0, 5.0), max_steer=0.5,
              max_accel=7.0, x0=None):
    """The sub-problem's KKT point to high accuracy (checker for the device solver)."""
    b = effective_box(CH, max_steer, max_accel)
    if x0 is None:
        x0 = np.zeros(2 * CH)
        if last is not None:
            x0[:2] = last
    args = (state, ref, last, N, CH, dt, L, Q, R, Qf)
    res = minimize(lambda x: objective(x, *args[:7], Q=Q, R=R, Qf=Qf), np.clip(x0, -b, b),
                   jac=lambda x: _grad(x, *args), method="L-BFGS-B", bounds=list(zip(-b, b)),
                   options={"maxiter": 10000, "ftol": 1e-16, "gtol": 1e-12, "maxcor": 50})
    return res.x.reshape(CH, 2), float(res.fun)


def track(wp, init, N=10, CH=5, dt=0.01, total_time=None, L=2.8):
    """PathTracker(...).run_simulation (:418-523): (times, states, controls, per-step SLSQP results)."""
    init = np.array(init, dtype=np.float64)
    if init[2] < -2.8:
        init[2] += 2 * np.pi
    ip = Interp(np.asarray(wp, dtype=np.float64), init)
    s = np.array([init[0], init[1], init[2], np.sqrt(np.sum(init[-2:] ** 2))])
    T = float(wp[-1, 2]) if total_time is None else total_time
    times, states, controls, last = [0.0], [s.copy()], [], None
    for k in range(int(T / dt)):
        tc = k * dt
        ref = np.zeros((N + 1, 2))
        prev = 0.0
        for i in range(N + 1):  # :464-478
            tr = tc + i * dt
            vx, vy = ip.reference(tr)[2:4]
            vr = np.sqrt(vx ** 2 + vy ** 2)
            th = ip.heading(tr) if vr >= 0.1 else prev
            prev = th
            ref[i] = [th, vr]
        useq, res = slsqp_solve(s, ref, last, N, CH, dt, L)
        if res.success:
            last = useq[0].copy()
        s = s + dynamics(s, useq[0], L) * dt
        states.append(s.copy())
        controls.append(useq[0].copy())
        times.append(tc + dt)
    return np.array(times), np.array(states), np.array(controls)
