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
