// cvae_loss.h — standalone conditional_vae_loss (Training_VAE.py:229-268), forward only.
//
// For callers that hold (recon, x_rel, mu, logvar) themselves (evaluation,
// the reference's loss API).  The training path never uses it: there the loss
// and dL/drecon are fused into the row-chain kernel's last epilogue.
// Pass 1: one workgroup per 32 rows writes 5 partial sums; pass 2 (one thread,
// fixed order, deterministic) forms the means exactly like finish_loss.
#pragma once
#include "cvae_device.h"
#include "cvae_wgrad.h"

__global__ __launch_bounds__(CVAE_THREADS) void loss_partial_kernel(const float* __restrict__ r,
                                                                    const float* __restrict__ x,
                                                                    const float* __restrict__ mu,
                                                                    const float* __restrict__ lv, int B, int S,
                                                                    int D, int Z, float* partials) {
  __shared__ float part[CVAE_NW * 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int b0 = blockIdx.x * 32, nrows = min(32, B - b0), I = S * D;
  float s_recon = 0.f, s_kl = 0.f, s_start = 0.f, s_t0 = 0.f, s_relu = 0.f;
  for (int e = tid; e < nrows * I; e += CVAE_THREADS) {
    const int row = e / I, col = e - row * I, s = col / D, d = col - s * D;
    const size_t o = (size_t)(b0 + row) * I + col;
    const float rv = r[o], diff = rv - x[o];
    s_recon += diff * diff;                                  // mse_loss(recon, x)   :240
    if (s == 0 && (d == 1 || d == 2)) s_start += diff * diff;  // start point         :250-252
    if (d == 0) {
      if (s == 0) s_t0 += rv * rv;                           // time starts at 0     :258
      if (s < S - 1) s_relu += fmaxf(rv - r[o + D], 0.f);    // relu(-(t_{s+1}-t_s)) :261-262
    }
  }
  for (int e = tid; e < nrows * Z; e += CVAE_THREADS) {
    const size_t o = (size_t)b0 * Z + e;
    s_kl += 1.f + lv[o] - mu[o] * mu[o] - expf(lv[o]);       // :243
  }
  s_recon = wave_sum(s_recon); s_kl = wave_sum(s_kl); s_start = wave_sum(s_start);
  s_t0 = wave_sum(s_t0); s_relu = wave_sum(s_relu);
  if (lane == 0) {
    part[wave * 8 + 0] = s_recon; part[wave * 8 + 1] = s_kl; part[wave * 8 + 2] = s_start;
    part[wave * 8 + 3] = s_t0; part[wave * 8 + 4] = s_relu;
  }
  __syncthreads();
  if (tid < 5) {
    float s = 0.f;
    for (int w = 0; w < CVAE_NW; ++w) s += part[w * 8 + tid];
    partials[blockIdx.x * 8 + tid] = s;
  }
}

__global__ void loss_finish_kernel(LossArgs la, int S, int D, int Z) {
  if (threadIdx.x < 64) finish_loss(la, S, D, Z);
}

// Backward of conditional_vae_loss (autograd of Training_VAE.py:240-267, the formulas of SURVEY
// §8a-a9 the fused loss epilogue uses, with the upstream gradients g[5] of (total, recon, kld,
// start, time) folded into per-term coefficients: c_term = g_total·w_term + g_term).  One thread per
// (row, s, d) element of recon plus one per (row, j) latent; elementwise and HBM-bound.
__global__ __launch_bounds__(CVAE_THREADS) void loss_backward_kernel(
    const float* __restrict__ r, const float* __restrict__ x, const float* __restrict__ mu,
    const float* __restrict__ lv, int B, int S, int D, int Z, cvae_loss_weights w, const float* __restrict__ g,
    float* __restrict__ d_recon, float* __restrict__ d_mu, float* __restrict__ d_lv) {
  const float g0 = g[0];
  const float c_r = g0 * w.recon + g[1];
  const float c_k = g0 * w.kld + g[2];
  const float c_s = w.start > 0.f ? g0 * w.start + g[3] : 0.f;  // :247 — the term is absent otherwise
  const float c_t = w.time > 0.f ? g0 * w.time + g[4] : 0.f;    // :256
  const int I = S * D;
  const float Bf = (float)B;
  const float inv_BSD = 1.f / (Bf * (float)I), inv_2B = 1.f / (2.f * Bf), inv_B = 1.f / Bf;
  const float inv_BS1 = S > 1 ? 1.f / (Bf * (float)(S - 1)) : 0.f, inv_BZ = 1.f / (Bf * (float)Z);
  const int64_t n_r = (int64_t)B * I, n_z = (int64_t)B * Z;
  for (int64_t e = (int64_t)blockIdx.x * CVAE_THREADS + threadIdx.x; e < n_r + n_z;
       e += (int64_t)gridDim.x * CVAE_THREADS) {
    if (e < n_r) {
      const int col = (int)(e % I), s = col / D, d = col - s * D;
      const float rv = r[e], diff = rv - x[e];
      float gi = c_r * 2.f * diff * inv_BSD;                                   // mse_loss   :240
      if (s == 0 && (d == 1 || d == 2) && w.start > 0.f) gi += c_s * 2.f * diff * inv_2B;  // :250-252
      if (d == 0 && w.time > 0.f) {
        if (s == 0) gi += c_t * 2.f * rv * inv_B;                             // :258
        if (s < S - 1 && rv - r[e + D] > 0.f) gi += c_t * inv_BS1;            // relu(r_s - r_s+1) :261-262
        if (s > 0 && r[e - D] - rv > 0.f) gi -= c_t * inv_BS1;
      }
      d_recon[e] = gi;
    } else {
      const int64_t k = e - n_r;
      d_mu[k] = c_k * mu[k] * inv_BZ;                                          // kld  :243
      d_lv[k] = c_k * 0.5f * (expf(lv[k]) - 1.f) * inv_BZ;
    }
  }
}

// Philox / Adam scalar checks (cvae_adam_scalars): the device's per-step Adam scalars for t = 1..n
__global__ void adam_scalars_kernel(double lr, double b1, double b2, int64_t n, float* out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    float a, b;
    adam_scalars(lr, b1, b2, (double)(t + 1), a, b);
    out[2 * t] = a;
    out[2 * t + 1] = b;
  }
}
