// cvae_mpc.h — batched MPC path tracking (MPC/MPC_Tracking.py): the step after
// generation, where every generated trajectory is tracked by a kinematic-bicycle MPC.
//
// The reference tracks ONE trajectory per process: a Python loop over time steps, each solving a
// 2·control_horizon-variable box-constrained NLP with scipy SLSQP and finite-difference gradients
// (MPC_Tracking.py:311-415).  Here one 64-lane wavefront owns one trajectory for the whole run,
// and the batch of trajectories is the grid:
//
//   prologue  PathInterpolator (:89-222): lanes 0-3 fit the x(t), y(t), vx(t), vy(t) splines
//             (scipy interp1d 'cubic' = not-a-knot, 'quadratic' = the parabola through 3 points,
//             'linear'), the start heading and the end velocity (the 1 ms heading scan :207-218,
//             64 instants per pass);
//   per step  the reference [theta, v] horizon (:464-478, lane k = horizon point k), then the MPC
//             problem solved to its KKT point by projected Newton: exact gradient and Hessian of
//             the tracking + control-increment cost through the Euler bicycle rollout (lane k =
//             time step for the rollout and its adjoint sums, lane j = decision variable for the
//             Hessian rows, the Cholesky and the solves, all in LDS), Armijo backtracking along
//             the projection onto the bounds; then the plant update (:484-486) with the first
//             control.
//
// Bounds follow the reference literally: SLSQP gets `bounds` listing control_horizon accel
// bounds then control_horizon steer bounds over the FLAT [a0, d0, a1, d1, ...] vector, plus the
// inequality constraints |a_i| <= max_accel, |d_i| <= max_steer; the feasible box is their
// intersection (flat index f < control_horizon: max_accel, else max_steer, intersected with the
// variable's own limit) — e.g. a_3, a_4 are held to +-0.5 at control_horizon 5.
//
// Everything is float64, like the reference.  The optimiser differs from SLSQP (which stops at
// ftol 1e-6 with finite-difference gradients): parity with the reference is stated as a
// tolerance on the closed loop and as "the KKT point's cost <= SLSQP's cost" per sub-problem.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#if CVAE_DIAG_MPC  // diagnostic build only: per-phase cycle totals of lane 0 (global vector atomics)
__device__ unsigned long long mpc_prof[8];
#define MPC_TIC() long long mpc_t_ = (long long)__builtin_readcyclecounter()
#define MPC_TOC(k)                                                                               \
  do {                                                                                           \
    const long long n_ = (long long)__builtin_readcyclecounter();                               \
    if (threadIdx.x == 0) atomicAdd(&mpc_prof[k], (unsigned long long)(n_ - mpc_t_));           \
    mpc_t_ = n_;                                                                                 \
  } while (0)
#else
#define MPC_TIC() ((void)0)
#define MPC_TOC(k) ((void)0)
#endif

constexpr int MPC_MAXWP = 64;   // waypoints per trajectory
constexpr int MPC_MAXH = 63;    // prediction horizon (N + 1 <= 64 lanes)
constexpr int MPC_MAXCH = 32;   // control horizon (2·CH <= 64 lanes)

struct MpcCfg {
  double L, max_steer, max_accel, dt;
  double q_th, q_v, qf_th, qf_v, r_a, r_d;
  double tol;
  int N, CH, max_iter, pad_;
};

// ---------------------------------------------------------------------------------------------
// wave helpers (one wavefront = one trajectory / problem; blockDim.x == 64)
__device__ __forceinline__ double mpc_wsum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double mpc_wmax(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double mpc_scan_incl(double v, int lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const double t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}
__device__ __forceinline__ void mpc_sync() { __syncthreads(); }  // one-wave workgroup

// the reference's heading convention (:202, :211, :273): theta if theta >= -2.8 else theta + 2*pi
__device__ __forceinline__ double mpc_wrap(double th) { return th >= -2.8 ? th : th + 2.0 * M_PI; }

// ---------------------------------------------------------------------------------------------
// PathInterpolator: four piecewise cubics (x, y over the waypoint times; vx, vy over t_vel)
struct MpcSpline {
  double tk[MPC_MAXWP];                 // waypoint times
  double tv[MPC_MAXWP];                 // velocity sample times [0, t[:-1] + dt/2]
  double c[4][MPC_MAXWP - 1][4];        // curve, interval, (c0, c1, c2, c3) in powers of (t - knot)
  double dat[4][MPC_MAXWP];             // fit inputs
  double start_theta, end_vx, end_vy, end_theta, end_x, end_y, t_end;
  int n, ok;
};


// fit curve `cv` through (kn[i], y[i]), i < n, with interp1d's kind for n points; tmp = 5·MPC_MAXWP
// doubles of this lane's scratch
__device__ void mpc_fit(MpcSpline& s, int cv, const double* kn, const double* y, int n, double* tmp) {
  double (*c)[4] = s.c[cv];
  if (n == 2) {  // 'linear'
    c[0][0] = y[0]; c[0][1] = (y[1] - y[0]) / (kn[1] - kn[0]); c[0][2] = 0.0; c[0][3] = 0.0;
    return;
  }
  if (n == 3) {  // 'quadratic': make_interp_spline(k=2) has no interior knot here = the parabola
    const double d01 = (y[1] - y[0]) / (kn[1] - kn[0]);
    const double d12 = (y[2] - y[1]) / (kn[2] - kn[1]);
    const double a2 = (d12 - d01) / (kn[2] - kn[0]);  // p(t) = y0 + d01 (t-t0) + a2 (t-t0)(t-t1)
    for (int i = 0; i < 2; ++i) {
      const double dx = kn[i] - kn[0];
      c[i][0] = i == 0 ? y[0] : y[0] + dx * (d01 + a2 * (kn[i] - kn[1]));
      c[i][1] = d01 + a2 * ((kn[i] - kn[0]) + (kn[i] - kn[1]));
      c[i][2] = a2;
      c[i][3] = 0.0;
    }
    return;
  }
  // 'cubic' (n >= 4): not-a-knot end conditions; the slopes m_i solve the tridiagonal system
  // scipy's CubicSpline assembles (elimination without pivoting); Hermite form per interval
  double* sub = tmp;
  double* dia = tmp + MPC_MAXWP;
  double* sup = tmp + 2 * MPC_MAXWP;
  double* rhs = tmp + 3 * MPC_MAXWP;
  double* m = tmp + 4 * MPC_MAXWP;
  auto h = [&](int i) { return kn[i + 1] - kn[i]; };
  auto sl = [&](int i) { return (y[i + 1] - y[i]) / h(i); };
  {
    const double d = kn[2] - kn[0];
    dia[0] = h(1); sup[0] = d; sub[0] = 0.0;
    rhs[0] = ((h(0) + 2.0 * d) * h(1) * sl(0) + h(0) * h(0) * sl(1)) / d;
  }
  for (int i = 1; i < n - 1; ++i) {
    sub[i] = h(i); dia[i] = 2.0 * (h(i - 1) + h(i)); sup[i] = h(i - 1);
    rhs[i] = 3.0 * (h(i) * sl(i - 1) + h(i - 1) * sl(i));
  }
  {
    const double d = kn[n - 1] - kn[n - 3];
    dia[n - 1] = h(n - 3); sub[n - 1] = d; sup[n - 1] = 0.0;
    rhs[n - 1] = (h(n - 2) * h(n - 2) * sl(n - 3) + (2.0 * d + h(n - 2)) * h(n - 3) * sl(n - 2)) / d;
  }
  for (int i = 1; i < n; ++i) {
    const double w = sub[i] / dia[i - 1];
    dia[i] -= w * sup[i - 1];
    rhs[i] -= w * rhs[i - 1];
  }
  m[n - 1] = rhs[n - 1] / dia[n - 1];
  for (int i = n - 2; i >= 0; --i) m[i] = (rhs[i] - sup[i] * m[i + 1]) / dia[i];
  for (int i = 0; i < n - 1; ++i) {
    const double hi = h(i), s0 = sl(i);
    const double t = (m[i] + m[i + 1] - 2.0 * s0) / hi;
    c[i][0] = y[i]; c[i][1] = m[i]; c[i][2] = (s0 - m[i]) / hi - t; c[i][3] = t / hi;
  }
}

// evaluate curve cv (knots kn, n points) at t; outside the knots the end pieces extrapolate
__device__ __forceinline__ double mpc_eval(const MpcSpline& s, int cv, const double* kn, int n, double t) {
  int lo = 0, hi = n - 2;  // the last i <= n-2 with kn[i] <= t (0 below the first knot)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (kn[mid] <= t) lo = mid; else hi = mid - 1;
  }
  const double* c = s.c[cv][lo];
  const double dx = t - kn[lo];
  return ((c[3] * dx + c[2]) * dx + c[1]) * dx + c[0];
}

// PathInterpolator.__init__ (:103-222) for waypoints wp[n][3] = (x, y, t) and the initial
// velocity (vx0, vy0); tmp = 4·5·MPC_MAXWP doubles of LDS scratch
__device__ void mpc_interp_init(MpcSpline& s, const double* wp, int n, double vx0, double vy0, int lane,
                                double* tmp) {
  if (lane < n) {
    s.tk[lane] = wp[lane * 3 + 2];
    s.dat[0][lane] = wp[lane * 3 + 0];
    s.dat[1][lane] = wp[lane * 3 + 1];
  }
  mpc_sync();
  if (lane < 2) mpc_fit(s, lane, s.tk, s.dat[lane], n, tmp + lane * 5 * MPC_MAXWP);
  mpc_sync();
  // velocity samples (:145-168): differences of the smoothed positions, at mid-interval times,
  // after the initial velocity at t = 0
  if (lane < n) {
    if (lane == 0) {
      s.tv[0] = 0.0;
      s.dat[2][0] = vx0;
      s.dat[3][0] = vy0;
    } else {
      const int i = lane - 1;
      double dt = s.tk[i + 1] - s.tk[i];
      dt = dt == 0.0 ? 1e-6 : dt;
      const double x1 = mpc_eval(s, 0, s.tk, n, s.tk[i + 1]), x0 = mpc_eval(s, 0, s.tk, n, s.tk[i]);
      const double y1 = mpc_eval(s, 1, s.tk, n, s.tk[i + 1]), y0 = mpc_eval(s, 1, s.tk, n, s.tk[i]);
      s.dat[2][lane] = (x1 - x0) / dt;
      s.dat[3][lane] = (y1 - y0) / dt;
      s.tv[lane] = s.tk[i] + dt / 2.0;
    }
  }
  mpc_sync();
  if (lane == 2 || lane == 3) mpc_fit(s, lane, s.tv, s.dat[lane], n, tmp + lane * 5 * MPC_MAXWP);
  mpc_sync();
  const double t_start = s.tk[0], t_end = s.tk[n - 1];
  const double st = mpc_wrap(atan2(mpc_eval(s, 3, s.tv, n, t_start), mpc_eval(s, 2, s.tv, n, t_start)));
  // end velocity (:204-218): if the wrapped heading at any instant of arange(0, t_end + 0.001,
  // 0.001) leaves start +- 45 deg, the velocity at the middle of the last interval, else at t_end
  const double step = 0.001;
  const int64_t cnt = (int64_t)ceil((t_end + step) / step);
  const double lim45 = 45.0 * M_PI / 180.0;
  bool hit = false;
  for (int64_t b = 0; b < cnt && !hit; b += 64) {
    const int64_t i = b + lane;
    bool h = false;
    if (i < cnt) {
      const double t1 = (double)i * step;
      const double th = mpc_wrap(atan2(mpc_eval(s, 3, s.tv, n, t1), mpc_eval(s, 2, s.tv, n, t1)));
      h = fabs(th - st) > lim45;
    }
    hit = __ballot(h) != 0ull;
  }
  const double te = hit ? (s.tk[n - 1] + s.tk[n - 2]) / 2.0 : t_end;
  const double evx = mpc_eval(s, 2, s.tv, n, te), evy = mpc_eval(s, 3, s.tv, n, te);
  if (lane == 0) {
    s.start_theta = st;
    s.end_vx = evx;
    s.end_vy = evy;
    s.end_theta = mpc_wrap(atan2(evy, evx));
    s.end_x = mpc_eval(s, 0, s.tk, n, t_end);
    s.end_y = mpc_eval(s, 1, s.tk, n, t_end);
    s.t_end = t_end;
    s.n = n;
  }
  mpc_sync();
}

// get_reference (:224-252) and get_reference_heading (:254-277) at time t
__device__ __forceinline__ void mpc_reference(const MpcSpline& s, double t, double& x, double& y, double& vx,
                                              double& vy, double& heading) {
  if (t <= s.t_end) {
    const int n = s.n;
    x = mpc_eval(s, 0, s.tk, n, t);
    y = mpc_eval(s, 1, s.tk, n, t);
    vx = mpc_eval(s, 2, s.tv, n, t);
    vy = mpc_eval(s, 3, s.tv, n, t);
    if (fabs(atan2(vy, vx) - s.start_theta) > 90.0 * M_PI / 180.0) {  // heading jump → end velocity
      vx = s.end_vx;
      vy = s.end_vy;
    }
    heading = mpc_wrap(atan2(vy, vx));
  } else {  // past the end: straight line at the end velocity, end heading
    const double de = t - s.t_end;
    x = s.end_x + s.end_vx * de;
    y = s.end_y + s.end_vy * de;
    vx = s.end_vx;
    vy = s.end_vy;
    heading = mpc_wrap(s.end_theta);
  }
}

// PathTracker.step's horizon (:464-478) for lane k <= N: (theta_ref_k, v_ref_k); a speed below 0.1
// keeps the previous point's heading (0.0 before the first valid one)
__device__ __forceinline__ void mpc_horizon(const MpcSpline& s, const MpcCfg& c, double t_cur, int lane,
                                            double& thr, double& vr) {
  double x, y, vx, vy, hd;
  const double t_ref = t_cur + (double)lane * c.dt;
  mpc_reference(s, t_ref, x, y, vx, vy, hd);
  vr = sqrt(vx * vx + vy * vy);
  const bool ok = lane <= c.N && vr >= 0.1;
  const unsigned long long m = __ballot(ok) & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
  const int src = m ? 63 - __clzll((long long)m) : 0;
  const double th = __shfl(hd, src, 64);
  thr = m ? th : 0.0;
}

// ---------------------------------------------------------------------------------------------
// The MPC sub-problem (MPCController.solve_mpc :311-415)
//
//   min_u  sum_{k=0..N} q_k^th (theta_k - theta_ref_k)^2 + q_k^v (v_k - v_ref_k)^2
//          + sum_i r_a (a_i - a_{i-1})^2 + r_d (d_i - d_{i-1})^2      (i = 0 against the last
//                                                                      control, if any)
//   v_{k+1} = v_k + a_{c(k)} dt,  theta_{k+1} = theta_k + v_k tan(d_{c(k)}) / L dt,  c(k) = min(k, CH-1)
//
// Variables in lane order: a_0..a_{CH-1}, d_0..d_{CH-1}.
struct MpcWs {
  double *u, *ut, *kv, *ktan, *G, *H;
  int ldh, ldg, kg;  // H row stride; G row stride (NV padded to 16) and rows (2(N+1) padded to 16)
};

constexpr int MPC_KPAD = 72;  // per-step arrays: 64 lanes + the 8-wide read-ahead of the G loop

__host__ __device__ inline int mpc_ldg(int CH) { return (2 * CH + 15) / 16 * 16; }
__host__ __device__ inline int mpc_kg(int N) { return (2 * (N + 1) + 15) / 16 * 16; }

__host__ __device__ inline size_t mpc_ws_doubles(int N, int CH) {
  const size_t nv = 2 * (size_t)CH;
  const size_t need = 4 * MPC_KPAD + (size_t)mpc_kg(N) * mpc_ldg(CH) + nv * (nv + 1);
  const size_t fit = 4 * 5 * MPC_MAXWP;  // spline-fit scratch reuses the region before the solver runs
  return need > fit ? need : fit;
}

__device__ __forceinline__ MpcWs mpc_ws(double* base, const MpcCfg& c) {
  const int nv = 2 * c.CH;
  MpcWs w;
  w.u = base; w.ut = base + MPC_KPAD; w.kv = base + 2 * MPC_KPAD; w.ktan = base + 3 * MPC_KPAD;
  w.ldg = mpc_ldg(c.CH);
  w.kg = mpc_kg(c.N);
  w.G = base + 4 * MPC_KPAD; w.H = w.G + w.kg * w.ldg; w.ldh = nv + 1;
  return w;
}

// the feasible half-width of variable j: SLSQP's bounds (flat index f < CH: max_accel, else
// max_steer) intersected with the inequality constraints of the variable's kind (:376-394)
__device__ __forceinline__ double mpc_bound(const MpcCfg& c, int j) {
  const bool is_a = j < c.CH;
  const int i = is_a ? j : j - c.CH;
  const int flat = 2 * i + (is_a ? 0 : 1);
  const double b = flat < c.CH ? c.max_accel : c.max_steer;
  return fmin(b, is_a ? c.max_accel : c.max_steer);
}

// #{i' < i : c(i') = j}: how many rollout steps before step i applied control j
__device__ __forceinline__ int mpc_cnt(int j, int i, int CH) { return j < CH - 1 ? (i > j ? 1 : 0) : (i > j ? i - j : 0); }

typedef double mpc_f64x4 __attribute__((ext_vector_type(4)));

struct MpcEval {
  double J, v, tn, eth, ev;
};

// cost at u (LDS, NV entries); lane k <= N returns its rollout state and residuals
__device__ MpcEval mpc_cost(const MpcCfg& c, const double* u, double th0, double v0, double thr, double vr,
                            bool has_last, double la, double ld, int lane) {
  const int N = c.N, CH = c.CH, NV = 2 * CH;
  const int ci = lane < CH ? lane : CH - 1;
  const double a = u[ci], tn = tan(u[CH + ci]);
  const double iv = lane < N ? a * c.dt : 0.0;
  const double v = v0 + (mpc_scan_incl(iv, lane) - iv);
  const double it = lane < N ? (v * tn / c.L) * c.dt : 0.0;
  const double th = th0 + (mpc_scan_incl(it, lane) - it);
  MpcEval e;
  e.v = v; e.tn = tn; e.eth = 0.0; e.ev = 0.0;
  double J = 0.0;
  if (lane <= N) {
    e.eth = th - thr;
    e.ev = v - vr;
    J = (lane < N ? c.q_th : c.qf_th) * e.eth * e.eth + (lane < N ? c.q_v : c.qf_v) * e.ev * e.ev;
  }
  if (lane < NV) {
    const bool isa = lane < CH;
    const int i = isa ? lane : lane - CH;
    if (i > 0 || has_last) {
      const double p = i > 0 ? u[lane - 1] : (isa ? la : ld);
      const double dd = u[lane] - p;
      J += (isa ? c.r_a : c.r_d) * dd * dd;
    }
  }
  e.J = mpc_wsum(J);
  return e;
}

// Gradient (returned per variable lane) and the Hessian's lower triangle (LDS) at the point e was
// evaluated at; exact = with the second-order terms of theta_k (Newton), else Gauss-Newton.
//
// With E_k = sum_{k' > k} 2 q_th,k' (theta_k' - ref) and P_k = 2 q_v,k (v_k - ref) + dt/L tan_k E_k
// (lane k), the adjoint sums collapse to wave scans:
//   dJ/da_j = dt sum_{i > j} P_i              (j < CH-1)     dt sum_{i >= CH} (i-CH+1) P_i  (j = CH-1)
//   dJ/dd_m = dt/L sec^2 d_m v_m E_m          (m < CH-1)     dt/L sec^2 d_m sum_{i >= CH-1} v_i E_i
// and likewise the second-order terms; the Gauss-Newton block is one MFMA product over the
// stacked Jacobian [dtheta/du; dv/du].
__device__ double mpc_system(const MpcCfg& c, const MpcWs& w, const MpcEval& e, int lane, bool has_last, double la,
                             double ld, bool exact) {
  const int N = c.N, CH = c.CH, NV = 2 * CH;
  const double dt = c.dt, kL = c.dt / c.L;
  const bool on = lane <= N;
  const double wt = lane < N ? 2.0 * c.q_th : 2.0 * c.qf_th, wv = lane < N ? 2.0 * c.q_v : 2.0 * c.qf_v;
  const double ae = on ? wt * e.eth : 0.0;
  const double inE = mpc_scan_incl(ae, lane);
  const double E = __shfl(inE, 63, 64) - inE;
  const double P = on ? wv * e.ev + kL * e.tn * E : 0.0;
  const double inP = mpc_scan_incl(P, lane);
  const double SP = __shfl(inP, 63, 64) - inP;                        // sum_{i > lane} P_i
  const double VE = e.v * E;
  const bool tail = lane >= CH - 1 && lane < N;                         // steps applying the last control
  const double TP = mpc_wsum(lane >= CH && on ? (double)(lane - CH + 1) * P : 0.0);
  const double S1 = mpc_wsum(tail ? E : 0.0);
  const double S2 = mpc_wsum(tail ? (double)(lane - CH + 1) * E : 0.0);
  const double S3 = mpc_wsum(tail ? VE : 0.0);
  w.kv[lane] = e.v;
  w.ktan[lane] = e.tn;
  const bool isa = lane < CH;
  const int vi = isa ? lane : lane - CH;  // index within the variable's kind
  const int src = lane < NV ? vi : 0;
  const double Em = __shfl(E, src, 64), VEm = __shfl(VE, src, 64);
  const double tsrc = __shfl(e.tn, src, 64);  // tan d_m = the tan step m applied (m <= CH-1 <= N-1)
  const double tm = lane < NV && !isa ? tsrc : 0.0, s2 = 1.0 + tm * tm;
  double g = 0.0;
  if (lane < NV) {
    if (isa) g = dt * (vi < CH - 1 ? SP : TP);
    else g = kL * s2 * (vi < CH - 1 ? VEm : S3);
    const double r2 = 2.0 * (isa ? c.r_a : c.r_d);
    if (vi > 0 || has_last) g += r2 * (w.u[lane] - (vi > 0 ? w.u[lane - 1] : (isa ? la : ld)));
    if (vi + 1 < CH) g -= r2 * (w.u[lane + 1] - w.u[lane]);
  }
  mpc_sync();
  // Jacobian rows into G: row k = dtheta_k/du (k = 0..N), row N+1+k = dv_k/du; zero padding to
  // kg rows x ldg columns (the MFMA tiles read whole 16 x 4 blocks)
  if (lane < w.ldg) {
    const int j = lane;
    const bool ja = j < CH, jd = !ja && j < NV;
    const int m = j - CH;
    const double s2j = jd ? s2 : 0.0;
    double gt = 0.0;
    w.G[j] = 0.0;
    w.G[(N + 1) * w.ldg + j] = 0.0;
    for (int k0 = 0; k0 < N; k0 += 8) {
      double tk[8], vk[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        tk[q] = w.ktan[k0 + q];
        vk[q] = w.kv[k0 + q];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = k0 + q;
        if (k < N) {
          double gv = 0.0;
          if (ja) {
            gt += kL * tk[q] * (dt * (double)mpc_cnt(j, k, CH));
            gv = dt * (double)mpc_cnt(j, k + 1, CH);
          } else if (jd && (k < CH - 1 ? k : CH - 1) == m) {
            gt += kL * vk[q] * s2j;
          }
          w.G[(k + 1) * w.ldg + j] = gt;
          w.G[(N + 2 + k) * w.ldg + j] = gv;
        }
      }
    }
    for (int r = 2 * (N + 1); r < w.kg; ++r) w.G[r * w.ldg + j] = 0.0;
  }
  mpc_sync();
  // Gauss-Newton block: H = G^T diag(2q) G with v_mfma_f64_16x16x4_f64 over the lower block
  // triangle.  A[i][k] = G[4s + k][16J + i], B[k][j] = w_k G[4s + k][16M + j]; D[row (l>>4) + 4r][col l&15].
  {
    const int nb = (NV + 15) / 16, kr = lane >> 4, cl = lane & 15;
    for (int J = 0; J < nb; ++J) {
      for (int M = 0; M <= J; ++M) {
        mpc_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int s16 = 0; s16 < w.kg; s16 += 16) {
          double a[4], b[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = s16 + 4 * q + kr;
            a[q] = w.G[r * w.ldg + 16 * J + cl];
            b[q] = w.G[r * w.ldg + 16 * M + cl];
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = s16 + 4 * q + kr;
            const double wr = r <= N ? (r < N ? 2.0 * c.q_th : 2.0 * c.qf_th)
                                     : (r - (N + 1) < N ? 2.0 * c.q_v : 2.0 * c.qf_v);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], wr * b[q], acc, 0, 0, 0);
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = 16 * J + kr + 4 * q, m = 16 * M + cl;
          if (i < NV && m <= i) w.H[i * w.ldh + m] = acc[q];
        }
      }
    }
  }
  mpc_sync();
  // second-order terms of theta_k (Newton) and the control-increment block, lower triangle
  if (lane < NV) {
    const double r2 = 2.0 * (isa ? c.r_a : c.r_d);
    double* hrow = w.H + lane * w.ldh;
    if (exact && !isa) {
      // d2/(dd_m da_j): dt/L sec^2 d_m dt sum_{i: c(i)=m} cnt_j(i) E_i
      const double base = kL * s2 * dt;
      for (int j = 0; j < CH; ++j) {
        const double so = vi < CH - 1 ? (vi > j ? Em : 0.0) : (j < CH - 1 ? S1 : S2);
        hrow[j] += base * so;
      }
      // d2/dd_m^2: dt/L 2 sec^2 tan sum_{i: c(i)=m} v_i E_i
      hrow[lane] += kL * 2.0 * s2 * tm * (vi < CH - 1 ? VEm : S3);
    }
    hrow[lane] += r2 * (double)((vi > 0 || has_last ? 1 : 0) + (vi + 1 < CH ? 1 : 0));
    if (vi > 0) hrow[lane - 1] -= r2;
  }
  mpc_sync();
  return g;
}

// Cholesky of the NV x NV matrix in w.H (lower triangle, in place); false if not positive
// definite.  Right-looking; the trailing update of step k is spread over all lanes by (i, j) pair.
__device__ bool mpc_cholesky(const MpcWs& w, int NV, int lane) {
  double dmax = lane < NV ? fabs(w.H[lane * w.ldh + lane]) : 0.0;
  dmax = mpc_wmax(dmax);
  const double tiny = 1e-13 * dmax;
  for (int k = 0; k < NV; ++k) {
    const double piv = w.H[k * w.ldh + k];
    if (!(piv > tiny)) return false;  // uniform: every lane read the same pivot
    const double lkk = sqrt(piv), inv = 1.0 / lkk;
    if (lane > k && lane < NV) w.H[lane * w.ldh + k] *= inv;
    if (lane == k) w.H[k * w.ldh + k] = lkk;
    mpc_sync();
    const int n = NV - 1 - k, T = n * (n + 1) / 2;
    for (int p0 = 0; p0 < T; p0 += 4 * 64) {
      int ii[4], jj[4];
      double hij[4], lik[4], ljk[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = p0 + q * 64 + lane;
        int r = (int)((sqrtf(8.0f * (float)p + 1.0f) - 1.0f) * 0.5f);
        if ((r + 1) * (r + 2) / 2 <= p) ++r;
        if (r * (r + 1) / 2 > p) --r;
        const bool ok = p < T;
        ii[q] = ok ? k + 1 + r : k;
        jj[q] = ok ? k + 1 + (p - r * (r + 1) / 2) : k;
        hij[q] = w.H[ii[q] * w.ldh + jj[q]];
        lik[q] = w.H[ii[q] * w.ldh + k];
        ljk[q] = w.H[jj[q] * w.ldh + k];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (p0 + q * 64 + lane < T) w.H[ii[q] * w.ldh + jj[q]] = hij[q] - lik[q] * ljk[q];
    }
    mpc_sync();
  }
  return true;
}

// solve L L^T x = b (b per lane, returned per lane)
__device__ double mpc_chol_solve(const MpcWs& w, int NV, int lane, double b) {
  const double dinv = lane < NV ? 1.0 / w.H[lane * w.ldh + lane] : 0.0;
  for (int k = 0; k < NV; ++k) {
    const double lik = lane > k && lane < NV ? w.H[lane * w.ldh + k] : 0.0;
    const double yk = __shfl(b * dinv, k, 64);
    if (lane == k) b = yk;
    else b -= lik * yk;
  }
  for (int k = NV - 1; k >= 0; --k) {
    const double lki = lane < k ? w.H[k * w.ldh + lane] : 0.0;
    const double xk = __shfl(b * dinv, k, 64);
    if (lane == k) b = xk;
    else b -= lki * xk;
  }
  return b;
}

// projected Newton on the box (Bertsekas 1982): Newton step on the variables not held at a bound
// by their gradient, Armijo backtracking along the projection arc.  Writes u (LDS); returns the
// iteration count; J = the cost at u.
__device__ int mpc_solve(const MpcCfg& c, const MpcWs& w, double th0, double v0, double thr, double vr, bool has_last,
                         double la, double ld, int lane, double& J) {
  const int CH = c.CH, NV = 2 * CH;
  const double b = lane < NV ? mpc_bound(c, lane) : 0.0;
  double uj = 0.0;  // the reference's initial guess: [last_control, 0, ...], inside the bounds
  if (has_last && lane == 0) uj = la;
  if (has_last && lane == CH) uj = ld;
  uj = fmin(fmax(uj, -b), b);
  if (lane < NV) w.u[lane] = uj;
  mpc_sync();
  MPC_TIC();
  MpcEval e = mpc_cost(c, w.u, th0, v0, thr, vr, has_last, la, ld, lane);
  MPC_TOC(1);
  int it = 0;
  bool exact = true;
  double lambda = 0.0;
  while (it < c.max_iter) {
    const double g = mpc_system(c, w, e, lane, has_last, la, ld, exact);
    MPC_TOC(2);
    const double pgj = lane < NV ? fabs(fmin(fmax(uj - g, -b), b) - uj) : 0.0;
    const double pg = mpc_wmax(pgj);
    if (pg <= c.tol) break;
    ++it;
    // variables held at a bound by their gradient
    const double eps = fmin(pg, 1e-3);
    const bool act = lane < NV && ((uj <= -b + eps && g > 0.0) || (uj >= b - eps && g < 0.0));
    const unsigned long long amask = __ballot(act);
    // held variables take a diagonally scaled gradient step (onto their bound after projection)
    const double hjj = lane < NV ? w.H[lane * w.ldh + lane] : 1.0;
    if (lane < NV) {
      for (int m = 0; m < NV; ++m) {
        const bool am = (amask >> m) & 1ull;
        if (act || am) w.H[lane * w.ldh + m] = m == lane ? 1.0 : 0.0;
        else if (m == lane) w.H[lane * w.ldh + m] += lambda;
      }
    }
    mpc_sync();
    const bool pd = mpc_cholesky(w, NV, lane);
    MPC_TOC(3);
    if (!pd) {  // indefinite: Gauss-Newton, then growing damping
      if (exact) exact = false;
      else lambda = lambda == 0.0 ? 1e-10 : lambda * 100.0;
      continue;
    }
    const double d = mpc_chol_solve(w, NV, lane, lane >= NV ? 0.0 : act ? -g / fmax(hjj, 1e-12) : -g);
    MPC_TOC(4);
    double alpha = 1.0;
    bool accepted = false;
    MpcEval et;
    for (int ls = 0; ls < 40; ++ls) {
      const double ut = lane < NV ? fmin(fmax(uj + alpha * d, -b), b) : 0.0;
      if (lane < NV) w.ut[lane] = ut;
      mpc_sync();
      et = mpc_cost(c, w.ut, th0, v0, thr, vr, has_last, la, ld, lane);
      const double dec = mpc_wsum(lane < NV ? g * (ut - uj) : 0.0);
      if (et.J <= e.J + 1e-4 * dec) {
        const double moved = mpc_wmax(fabs(ut - uj));
        uj = ut;
        accepted = moved > 0.0;
        break;
      }
      alpha *= 0.5;
    }
    MPC_TOC(1);
    if (!accepted) {
      if (exact) {  // the Newton model misled the search: retry from here with Gauss-Newton
        exact = false;
        continue;
      }
      break;
    }
    if (lane < NV) w.u[lane] = uj;
    mpc_sync();
    const bool stalled = !(e.J - et.J > 1e-15 * fabs(e.J));  // no representable progress left
    e = et;
    lambda = 0.0;
    const bool full = alpha == 1.0;
    if (stalled && (full || !exact)) break;  // converged (or Gauss-Newton cannot progress either)
    exact = full;  // after a backtracked step take the Gauss-Newton model once
  }
  J = e.J;
  return it;
}

// plant update (:484-486, VehicleModel.dynamics :39-64): clip, bicycle derivative, Euler step
__device__ __forceinline__ void mpc_plant(const MpcCfg& c, double* st, double a, double dl) {
  a = fmin(fmax(a, -c.max_accel), c.max_accel);
  dl = fmin(fmax(dl, -c.max_steer), c.max_steer);
  const double x = st[0], y = st[1], th = st[2], v = st[3];
  const double dx = v * cos(th), dy = v * sin(th), dth = v * tan(dl) / c.L;
  st[0] = x + dx * c.dt;
  st[1] = y + dy * c.dt;
  st[2] = th + dth * c.dt;
  st[3] = v + a * c.dt;
}

// ---------------------------------------------------------------------------------------------
// kernels: one 64-lane workgroup per trajectory / problem

// PathTracker(waypoints, initial_state).run_simulation over n_steps[p] steps for every path p.
// init[p] = (x, y, theta, vx, vy) with theta already wrapped (:435-436).  Outputs rows
// states[off[p] + p + s] (s = 0..n_steps), controls[off[p] + s] (s < n_steps); iters likewise.
__global__ __launch_bounds__(64) void mpc_track_kernel(MpcCfg c, const double* __restrict__ wp,
                                                       const int32_t* __restrict__ wp_off,
                                                       const double* __restrict__ init,
                                                       const int32_t* __restrict__ n_steps,
                                                       const int64_t* __restrict__ off, double* __restrict__ states,
                                                       double* __restrict__ controls, int32_t* __restrict__ iters) {
  extern __shared__ double mpc_smem[];
  MpcSpline& sp = *reinterpret_cast<MpcSpline*>(mpc_smem);
  double* wsbase = mpc_smem + (sizeof(MpcSpline) + 7) / 8;
  const int p = blockIdx.x, lane = threadIdx.x;
  const int n = wp_off[p + 1] - wp_off[p];
  const int ns = n_steps[p];
  double* srow = states + (off[p] + p) * 4;
  double* crow = controls + off[p] * 2;
  const double* ip = init + p * 5;
  if (n < 2 || n > MPC_MAXWP || ns < 0) {  // the host validates; never index out of the spline
    for (int64_t r = lane; r < (int64_t)(ns + 1) * 4; r += 64) srow[r] = __builtin_nan("");
    return;
  }
  mpc_interp_init(sp, wp + (int64_t)wp_off[p] * 3, n, ip[3], ip[4], lane, wsbase);
  const MpcWs w = mpc_ws(wsbase, c);
  double st[4] = {ip[0], ip[1], ip[2], sqrt(ip[3] * ip[3] + ip[4] * ip[4])};
  if (lane < 4) srow[lane] = st[lane];
  bool has_last = false;
  double la = 0.0, ld = 0.0;
  for (int s = 0; s < ns; ++s) {
    double thr, vr, J;
    MPC_TIC();
    mpc_horizon(sp, c, (double)s * c.dt, lane, thr, vr);
    MPC_TOC(0);
    const int it = mpc_solve(c, w, st[2], st[3], thr, vr, has_last, la, ld, lane, J);
    const double a = w.u[0], dl = w.u[c.CH];
    mpc_plant(c, st, a, dl);
    if (lane < 4) srow[(s + 1) * 4 + lane] = st[lane];
    if (lane < 2) crow[s * 2 + lane] = lane == 0 ? a : dl;
    if (iters && lane == 0) iters[off[p] + s] = it;
    has_last = true;
    la = a;
    ld = dl;
    mpc_sync();
  }
}

// independent sub-problems: state[p] = (x, y, theta, v), ref[p][k] = (theta_ref, v_ref), k <= N,
// last[p] = previous control or NaN (none).  u[p][i] = (a_i, d_i), i < CH.
__global__ __launch_bounds__(64) void mpc_solve_kernel(MpcCfg c, const double* __restrict__ state,
                                                       const double* __restrict__ ref, const double* __restrict__ last,
                                                       double* __restrict__ u, double* __restrict__ cost,
                                                       int32_t* __restrict__ iters) {
  extern __shared__ double mpc_smem[];
  const int p = blockIdx.x, lane = threadIdx.x;
  const MpcWs w = mpc_ws(mpc_smem, c);
  const double* r = ref + (int64_t)p * (c.N + 1) * 2;
  const double thr = lane <= c.N ? r[lane * 2] : 0.0, vr = lane <= c.N ? r[lane * 2 + 1] : 0.0;
  const double la = last[p * 2], ld = last[p * 2 + 1];
  const bool has_last = !(isnan(la) || isnan(ld));
  double J;
  const int it = mpc_solve(c, w, state[p * 4 + 2], state[p * 4 + 3], thr, vr, has_last, has_last ? la : 0.0,
                           has_last ? ld : 0.0, lane, J);
  if (lane < 2 * c.CH) {
    const int i = lane < c.CH ? lane : lane - c.CH;
    u[(int64_t)p * 2 * c.CH + 2 * i + (lane < c.CH ? 0 : 1)] = w.u[lane];
  }
  if (lane == 0) {
    cost[p] = J;
    if (iters) iters[p] = it;
  }
}

// PathInterpolator queries: out[p][i] = (x, y, vx, vy, heading) at t[i]; scal[p] = (start_theta,
// end_vx, end_vy, end_theta, end_x, end_y)
__global__ __launch_bounds__(64) void mpc_reference_kernel(const double* __restrict__ wp,
                                                           const int32_t* __restrict__ wp_off,
                                                           const double* __restrict__ init,
                                                           const double* __restrict__ t, int n_t,
                                                           double* __restrict__ out, double* __restrict__ scal) {
  extern __shared__ double mpc_smem[];
  MpcSpline& sp = *reinterpret_cast<MpcSpline*>(mpc_smem);
  double* tmp = mpc_smem + (sizeof(MpcSpline) + 7) / 8;
  const int p = blockIdx.x, lane = threadIdx.x;
  const int n = wp_off[p + 1] - wp_off[p];
  if (n < 2 || n > MPC_MAXWP) return;
  mpc_interp_init(sp, wp + (int64_t)wp_off[p] * 3, n, init[p * 5 + 3], init[p * 5 + 4], lane, tmp);
  for (int i = lane; i < n_t; i += 64) {
    double* o = out + ((int64_t)p * n_t + i) * 5;
    mpc_reference(sp, t[i], o[0], o[1], o[2], o[3], o[4]);
  }
  if (lane == 0) {
    double* q = scal + p * 6;
    q[0] = sp.start_theta; q[1] = sp.end_vx; q[2] = sp.end_vy; q[3] = sp.end_theta; q[4] = sp.end_x;
    q[5] = sp.end_y;
  }
}
