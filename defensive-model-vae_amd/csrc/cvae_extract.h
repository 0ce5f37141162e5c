// cvae_extract.h — Traj_Data_Process.process_csv (:72-122) for many parsed CSV logs at once
// (the step before training).  Parsing stays on the host (pandas.read_csv, as the
// reference); the per-file work — the scene's start row, the first later end row, the
// np.linspace resampling of the ego track and the time column — is one workgroup per file.
//
// Columns: [EX_NCOL][n_rows] float64 in the order of cvae_amd.preprocess.COLUMNS; file f owns rows
// [off[f], off[f+1]).  Every arithmetic step restates numpy's float64 operation and order (no FMA
// contraction: explicit __dmul_rn / __dadd_rn), so the outputs are bit-identical to the host path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

enum { EX_EGO_X = 0, EX_EGO_Y, EX_SV1_X, EX_SV1_Y, EX_SV1_VX, EX_SV1_VY, EX_SV1_YAW, EX_SV2_VX, EX_SV2_VY, EX_NCOL };
// scene ids (Traj_Data_Process.py:8-25 SCENE_CONFIG)
enum { EX_STATIC = 0, EX_DYNAMIC = 1, EX_PREDICTABLE = 2, EX_UNPREDICTABLE = 3 };

__device__ __forceinline__ double excol(const double* cols, int64_t n, int c, int64_t r) { return cols[c * n + r]; }

__device__ __forceinline__ bool ex_start(const double* cols, int64_t n, int64_t r, int scene) {
  const double ey = excol(cols, n, EX_EGO_Y, r);
  switch (scene) {
    case EX_STATIC:  // (ego_y >= 18) & (sv2_vx != 0) & (sv2_vy != 0)
      return ey >= 18.0 && excol(cols, n, EX_SV2_VX, r) != 0.0 && excol(cols, n, EX_SV2_VY, r) != 0.0;
    case EX_DYNAMIC:  // sv1_yaw < -170
      return excol(cols, n, EX_SV1_YAW, r) < -170.0;
    case EX_PREDICTABLE:  // (sv1_vx != 0) & (sv1_vy != 0) & (ego_y <= 40) & (ego_y != 0)
      return excol(cols, n, EX_SV1_VX, r) != 0.0 && excol(cols, n, EX_SV1_VY, r) != 0.0 && ey <= 40.0 && ey != 0.0;
    default: {  // (ego_x - sv1_x)**2 + (ego_y - sv1_y)**2 <= 40**2  &  sv1_yaw >= -89.9
      const double dx = excol(cols, n, EX_EGO_X, r) - excol(cols, n, EX_SV1_X, r);
      const double dy = ey - excol(cols, n, EX_SV1_Y, r);
      return __dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)) <= 1600.0 && excol(cols, n, EX_SV1_YAW, r) >= -89.9;
    }
  }
}

__device__ __forceinline__ bool ex_end(const double* cols, int64_t n, int64_t r, int scene) {
  switch (scene) {
    case EX_STATIC: return excol(cols, n, EX_EGO_Y, r) >= 95.0;
    case EX_DYNAMIC: return excol(cols, n, EX_EGO_X, r) < -186.0;
    case EX_PREDICTABLE: return excol(cols, n, EX_EGO_Y, r) <= -80.0;
    default: return excol(cols, n, EX_SV1_X, r) > 15.0 && excol(cols, n, EX_SV1_YAW, r) < -85.0;
  }
}

constexpr int EX_THREADS = 256;

// block-wide minimum of a row index (INT64_MAX = none)
__device__ __forceinline__ int64_t ex_block_min(int64_t v, int64_t* red) {
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t m = red[0];
  for (int k = 1; k < EX_THREADS / 64; ++k) m = red[k] < m ? red[k] : m;
  __syncthreads();
  return m;
}

// np.linspace(0, n - 1, P, dtype=int)[k]: float64 step (n-1)/(P-1), k·step, the last sample = n-1
__device__ __forceinline__ int64_t ex_linspace(int64_t n, int P, int k) {
  if (k == P - 1) return n - 1;
  const double step = (double)(n - 1) / (double)(P - 1);
  return (int64_t)__dmul_rn((double)k, step);
}

__global__ __launch_bounds__(EX_THREADS) void extract_kernel(const double* __restrict__ cols, int64_t n_rows,
                                                              const int64_t* __restrict__ off, int scene, int P,
                                                              int extend_mid, double time_interval,
                                                              double* __restrict__ out, int* __restrict__ valid) {
  __shared__ int64_t red[EX_THREADS / 64];
  const int f = blockIdx.x;
  const int64_t r0 = off[f], r1 = off[f + 1];
  // start row: the first row whose start condition holds (:76-83)
  int64_t s = INT64_MAX;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += EX_THREADS)
    if (ex_start(cols, n_rows, r, scene)) { s = r; break; }
  s = ex_block_min(s, red);
  double* o = out + (size_t)f * P * 3;
  if (s == INT64_MAX) {  // no start row → None
    if (threadIdx.x == 0) valid[f] = 0;
    return;
  }
  // end row: the first LATER row whose end condition holds; the track stops before it (:87-95)
  int64_t e = INT64_MAX;
  for (int64_t r = s + 1 + threadIdx.x; r < r1; r += EX_THREADS)
    if (ex_end(cols, n_rows, r, scene)) { e = r; break; }
  e = ex_block_min(e, red);
  const int64_t stop = e == INT64_MAX ? r1 : e;
  const int64_t n = stop - s;
  if (n < P) {  // fewer rows than target_points → None (:101-102)
    if (threadIdx.x == 0) valid[f] = 0;
    return;
  }
  if (threadIdx.x == 0) valid[f] = 1;
  for (int k = threadIdx.x; k < P; k += EX_THREADS) {
    int64_t i = ex_linspace(n, P, k);
    if (extend_mid && k > 0 && k < P - 1) {  // ceil((idx[k-1] + idx[k]) / 2) for the inner points (:109-114)
      const int64_t a = ex_linspace(n, P, k - 1), b = i;
      i = (int64_t)ceil((double)(a + b) / 2.0);
    }
    // arange(P) * time_interval * ((n - 1) / (P - 1))  (:117, numpy's left-to-right order)
    const double t = __dmul_rn(__dmul_rn((double)k, time_interval), (double)(n - 1) / (double)(P - 1));
    o[k * 3 + 0] = t;
    o[k * 3 + 1] = excol(cols, n_rows, EX_EGO_X, s + i);
    o[k * 3 + 2] = excol(cols, n_rows, EX_EGO_Y, s + i);
  }
}
