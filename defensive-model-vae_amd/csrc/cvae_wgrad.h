// cvae_wgrad.h — weight/bias gradients (a batch reduction) and the Adam update.
//
// wgrad_kernel: one workgroup per 32×32 tile of one layer's padded weight
// matrix.  dW_l[o][i] = Σ_b gT(l)[o][b] · xT(l)[i][b]  (dW = Gᵀ·X,
// K = batch), both operands batch-contiguous in the activation arena, MFMA
// 16x16x32 bf16 (or 4×16x16x4 f32) with the K range split over the 4 waves
// and combined through LDS in a fixed order (deterministic).  Tiles with
// i0 == 0 also reduce the bias gradient db = Σ_b G.
//
// The epilogue either writes the fp32 gradient into the flat state_dict-ordered
// buffer (data-parallel path: all-reduce comes next) or applies torch's Adam
// (torch/optim/adam.py _single_tensor_adam, replacing optimizer.step() at
// Training_VAE.py:363) in place and refreshes the padded operand copies
// Wf/Wb/bias that the row-chain kernel reads — the gradient never round-trips
// through HBM.  param_kernel does the same update from a gradient buffer
// (after the all-reduce) or just repacks the copies (PACK).
#pragma once
#include "cvae_device.h"

enum { PM_GRAD = 0, PM_ADAM = 1, PM_PACK = 2 };

// Diagnostic builds only: skip refreshing the operand copies after Adam (wrong results) to
// price the row-chain's cold weight reads.
#ifndef CVAE_DIAG_NOWPACK
#define CVAE_DIAG_NOWPACK 0
#endif

#ifndef CVAE_DIAG_STAMPS
#define CVAE_DIAG_STAMPS 0
#endif
#if CVAE_DIAG_STAMPS
// diagnostic builds only: [block][4] s_memrealtime at entry, after the MFMA loop, after the
// cross-wave reduction barrier, at exit
__device__ unsigned long long* g_wstamps;
#define WSTAMP(k)                                                                         \
  do {                                                                                    \
    if (threadIdx.x == 0 && g_wstamps) g_wstamps[blockIdx.x * 4 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define WSTAMP(k) do { } while (0)
#endif

struct AdamArgs {
  float* params;      // flat fp32 master (state_dict order)
  float* m;
  float* v;
  float* grads;       // PM_GRAD: output; param_kernel PM_ADAM: input
  float grad_scale;
  float lr_neg_step;  // -lr / (1 - beta1^t)
  float bc2_sqrt;     // sqrt(1 - beta2^t)
  float beta1_w;      // 1 - beta1  (lerp weight)
  float beta2;
  float one_m_beta2;
  float eps;
  int pad_;
};

struct LossArgs {
  const float* partials;  // [ntiles][8]
  int ntiles;
  int batch;
  float w_recon, w_kld, w_start, w_time;
  float* loss_out;        // [5] nullable
  float* loss_accum;      // [5] nullable, += loss * batch
};

__device__ __forceinline__ float adam_update(float p, float g, int64_t idx, const AdamArgs& a) {
  float m = a.m[idx], v = a.v[idx];
  // exp_avg.lerp_(grad, 1 - beta1): weight < 0.5 branch of at::lerp
  m = a.beta1_w < 0.5f ? m + a.beta1_w * (g - m) : g - (g - m) * (1.f - a.beta1_w);
  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
  v = v * a.beta2;
  v = v + a.one_m_beta2 * g * g;
  // denom = exp_avg_sq.sqrt() / bias_correction2_sqrt + eps;  param.addcdiv_(exp_avg, denom, -step_size)
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p + a.lr_neg_step * m / denom;
  a.m[idx] = m;
  a.v[idx] = v;
  return p;
}

// weight element (o, i) of layer L in padded coordinates; g valid for PM_GRAD / fused PM_ADAM
template <typename T, int MODE>
__device__ __forceinline__ void apply_weight(const LayerDev& L, int o, int i, float g, const AdamArgs& a) {
  if (o >= L.Np || i >= L.Kp) return;
  float w = 0.f;
  if (o < L.N && i < L.K) {
    const int seg = (L.nseg == 2 && o >= L.seg_rows0) ? 1 : 0;
    const int orow = seg ? o - L.seg_rows0 : o;
    const int64_t idx = L.pw[seg] + (int64_t)orow * L.K + i;
    if (MODE == PM_GRAD) { a.grads[idx] = g; return; }
    w = a.params[idx];
    if (MODE == PM_ADAM) {
      w = adam_update(w, g, idx, a);
      a.params[idx] = w;
    }
  } else if (MODE == PM_GRAD) {
    return;
  }
  if (CVAE_DIAG_NOWPACK && MODE == PM_ADAM) return;
  ((T*)L.Wf)[frag_off<T>(o, i, L.Kp)] = to_t<T>(w);  // forward operand: rows o, K = inputs
  ((T*)L.Wb)[frag_off<T>(i, o, L.Np)] = to_t<T>(w);  // dX operand (Wᵀ): rows i, K = outputs
}

template <int MODE>
__device__ __forceinline__ void apply_bias(const LayerDev& L, int o, float g, const AdamArgs& a) {
  if (o >= L.Np) return;
  float w = 0.f;
  if (o < L.N) {
    const int seg = (L.nseg == 2 && o >= L.seg_rows0) ? 1 : 0;
    const int64_t idx = L.pb[seg] + (seg ? o - L.seg_rows0 : o);
    if (MODE == PM_GRAD) { a.grads[idx] = g; return; }
    w = a.params[idx];
    if (MODE == PM_ADAM) {
      w = adam_update(w, g, idx, a);
      a.params[idx] = w;
    }
  } else if (MODE == PM_GRAD) {
    return;
  }
  if (CVAE_DIAG_NOWPACK && MODE == PM_ADAM) return;
  L.bias[o] = w;
}

// called by one whole wave: lane-strided partial sums, then a fixed-order butterfly (deterministic)
__device__ void finish_loss(const LossArgs& l, int S, int D, int Z) {
  const int lane = threadIdx.x & 63;
  float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int t = lane; t < l.ntiles; t += 64)
    for (int k = 0; k < 5; ++k) s[k] += l.partials[t * 8 + k];
  for (int k = 0; k < 5; ++k) s[k] = wave_sum(s[k]);
  if (lane != 0) return;
  const float B = (float)l.batch;
  const float recon = s[0] / (B * (float)(S * D));          // mse_loss mean   (:240)
  const float kld = -0.5f * s[1] / (B * (float)Z);          // (:243)
  const float start = l.w_start > 0.f ? s[2] / (2.f * B) : 0.f;  // (:246-252)
  const float time = l.w_time > 0.f ? s[3] / B + (S > 1 ? s[4] / (B * (float)(S - 1)) : 0.f) : 0.f;  // (:255-264)
  const float total = l.w_recon * recon + l.w_kld * kld + l.w_start * start + l.w_time * time;  // (:267)
  const float v[5] = {total, recon, kld, start, time};
  for (int k = 0; k < 5; ++k) {
    if (l.loss_out) l.loss_out[k] = v[k];
    if (l.loss_accum) l.loss_accum[k] += v[k] * B;
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(CVAE_THREADS) void wgrad_kernel(NetDev net, const TileDesc* __restrict__ tiles,
                                                             int Bk, AdamArgs aa, LossArgs la) {
  using V = typename Op<T>::V;
  constexpr int EPL = Op<T>::EPL, KC = Op<T>::KC;
  __shared__ __attribute__((aligned(16))) float red[CVAE_NW * 32 * 33];
  const TileDesc td = tiles[blockIdx.x];
  const LayerDev& L = net.L[td.layer];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int r16 = lane & 15, kq = (lane >> 4) * EPL;
  const int Bp = net.Bp;
  const T* G = (const T*)L.gT;
  const T* X = (const T*)L.xT;

  WSTAMP(0);
  if (blockIdx.x == 0 && tid < 64 && la.partials) finish_loss(la, net.S, net.D, net.Z);

  f32x4 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const T* gp[2];
  const T* xp[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) gp[m] = G + (size_t)(td.o0 + m * 16 + r16) * Bp + kq;
#pragma unroll
  for (int n = 0; n < 2; ++n) xp[n] = X + (size_t)(td.i0 + n * 16 + r16) * Bp + kq;
  // this wave's chunks: c = wave + CVAE_NW*j; PF chunks of loads kept in flight
  const int nk = Bk / KC;
  const int nmine = nk > wave ? (nk - wave + CVAE_NW - 1) / CVAE_NW : 0;
  constexpr int PF = 4;
  V ga[PF][2], xb[PF][2];
  auto load = [&](int u, int j) {  // unconditional, clamped to this wave's last chunk
    const int c = (wave + CVAE_NW * min(j, nmine > 0 ? nmine - 1 : 0)) * KC;
#pragma unroll
    for (int m = 0; m < 2; ++m) ga[u][m] = *(const V*)(gp[m] + c);
#pragma unroll
    for (int n = 0; n < 2; ++n) xb[u][n] = *(const V*)(xp[n] + c);
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) load(u, u);
  for (int j0 = 0; j0 < nmine; j0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int j = j0 + u;
      if (j < nmine) {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) acc[m][n] = mfma_chunk(ga[u][m], xb[u][n], acc[m][n]);
      }
      load(u, j + PF);
    }
  }
  WSTAMP(1);
  float* rw = red + wave * 32 * 33;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) rw[(m * 16 + (lane >> 4) * 4 + i) * 33 + n * 16 + r16] = acc[m][n][i];

  // bias gradient: 8 threads per output row, 16-B loads along the batch
  float db = 0.f;
  if (td.i0 == 0) {
    const int o = tid >> 3, part = tid & 7;
    const T* gr = G + (size_t)(td.o0 + o) * Bp;
#pragma unroll 4
    for (int c = part * EPL; c < Bk; c += 8 * EPL) {
      const V v = *(const V*)(gr + c);
#pragma unroll
      for (int e = 0; e < EPL; ++e) db += (float)v[e];
    }
    db += __shfl_xor(db, 1, 64);
    db += __shfl_xor(db, 2, 64);
    db += __shfl_xor(db, 4, 64);
  }
  __syncthreads();
  WSTAMP(2);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = q * CVAE_THREADS + tid;
    const int o = e >> 5, i = e & 31;
    float g = 0.f;
#pragma unroll
    for (int w = 0; w < CVAE_NW; ++w) g += red[w * 32 * 33 + o * 33 + i];
    apply_weight<T, MODE>(L, td.o0 + o, td.i0 + i, g, aa);
  }
  if (td.i0 == 0 && (tid & 7) == 0) apply_bias<MODE>(L, td.o0 + (tid >> 3), db, aa);
#if CVAE_DIAG_STAMPS
  __syncthreads();
  WSTAMP(3);
#endif
}

// Adam from a (reduced) gradient buffer, or repack of the operand copies.
template <typename T, int MODE>
__global__ __launch_bounds__(CVAE_THREADS) void param_kernel(NetDev net, const TileDesc* __restrict__ tiles,
                                                             AdamArgs aa) {
  const TileDesc td = tiles[blockIdx.x];
  const LayerDev& L = net.L[td.layer];
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = q * CVAE_THREADS + tid;
    const int o = td.o0 + (e >> 5), i = td.i0 + (e & 31);
    float g = 0.f;
    if (MODE == PM_ADAM && o < L.N && i < L.K) {
      const int seg = (L.nseg == 2 && o >= L.seg_rows0) ? 1 : 0;
      g = aa.grads[L.pw[seg] + (int64_t)(seg ? o - L.seg_rows0 : o) * L.K + i] * aa.grad_scale;
    }
    apply_weight<T, MODE>(L, o, i, g, aa);
  }
  if (td.i0 == 0 && tid < 32) {
    const int o = td.o0 + tid;
    float g = 0.f;
    if (MODE == PM_ADAM && o < L.N) {
      const int seg = (L.nseg == 2 && o >= L.seg_rows0) ? 1 : 0;
      g = aa.grads[L.pb[seg] + (seg ? o - L.seg_rows0 : o)] * aa.grad_scale;
    }
    apply_bias<MODE>(L, o, g, aa);
  }
}
