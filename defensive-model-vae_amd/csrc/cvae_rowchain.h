// cvae_rowchain.h — the fused per-row-tile training kernel.
//
// One workgroup (4 waves) owns R consecutive batch rows and runs, entirely in
// LDS/registers, the whole per-row part of the reference step
// (Training_VAE.py:345-362):
//   relative transform (:345-348) → condition_encoder (:132-137,:190) →
//   encoder (:141-151,:187) → cat + fc_mu‖fc_logvar (:193-196) →
//   reparameterize (:199-206) → decoder (:158-167,:214-215) →
//   conditional_vae_loss and dL/drecon (:229-268) → backward of every
//   activation (autograd of the above).
// Rows never interact, so no inter-workgroup communication is needed.  The
// weight gradients (a batch reduction) are left to cvae_wgrad.h: this kernel
// stores every layer input xT(l) and pre-activation gradient gT(l)
// feature-major into the activation arena.
//
// GEMM core: `dense` computes Y[R×Np] = X[R×Kp]·Wᵀ with X from LDS (A operand,
// ds_read_b128) and W streamed from L2 straight into registers (B operand, one
// 16-B global load per lane per K chunk, PF chunks in flight).  Each wave owns
// pairs of 16-column tiles; MFMA 16x16x32 bf16 or 4×16x16x4 f32 per chunk.
// ReLU masks are kept as bits in LDS for the backward pass.
#pragma once
#include "cvae_device.h"

enum { RC_TRAIN = 0, RC_FWD = 1, RC_DECODE = 2 };

// Diagnostic builds only (scripts/diag_rowchain.sh): drop the arena stores / bias loads to
// price them.  Results are wrong in those builds; the shipped library defines neither.
#ifndef CVAE_DIAG_NOSTORE
#define CVAE_DIAG_NOSTORE 0
#endif
#ifndef CVAE_DIAG_NOBIAS
#define CVAE_DIAG_NOBIAS 0
#endif

struct RowArgs {
  const void* x;          // (N_total, S, D) operand dtype
  const int64_t* idx;     // optional row gather
  int batch;
  int pad_;
  const float* eps;       // optional (batch, Z)
  uint64_t seed, offset;
  float w_recon, w_kld, w_start, w_time;
  float* partials;        // [gridDim.x][8] loss partial sums
  float* recon_out;       // FWD/DECODE outputs (fp32, nullable)
  float* mu_out;
  float* lv_out;
  float* hc_out;
  const float* z_in;      // DECODE inputs
  const float* start_in;  // DECODE, or FWD with x already relative
  const float* hc_in;     // DECODE: given condition features (skips the condition encoder)
  int x_relative;         // 1: x is relative, condition = start_in (no transform)
  int pad2_;
};

struct LdsPlan {
  int sx, sp, shc, sdec, scin;   // row strides (elements of T)
  int mw;                        // mask words per row
  int oXin, oP0, oP1, oHc, oDec, oCin, oMuLv, oEps, oStd, oDz, oU, oRch0, oGd0, oStart, oRow, oMask, oPart;
  int total;
};

__host__ __device__ inline int rup(int v, int a) { return (v + a - 1) / a * a; }

__host__ __device__ inline LdsPlan lds_plan(const NetDev& n, int R, int tsize) {
  LdsPlan p;
  const int pad = 16 / tsize;
  p.sx = n.Ip + pad;
  p.sp = (n.Hp > n.Zp2 ? n.Hp : n.Zp2) + pad;
  p.shc = n.Hcp + pad;
  p.sdec = n.ZHp + pad;
  p.scin = n.Cp + pad;
  p.mw = n.Hp / 32;
  const int nmask = 2 + n.n_enc + (n.n_dec - 1);
  int o = 0;
  auto take = [&](int bytes) { int r = o; o += rup(bytes, 16); return r; };
  p.oXin = take(R * p.sx * tsize);
  p.oP0 = take(R * p.sp * tsize);
  p.oP1 = take(R * p.sp * tsize);
  p.oHc = take(R * p.shc * tsize);
  p.oDec = take(R * p.sdec * tsize);
  p.oCin = take(R * p.scin * tsize);
  p.oMuLv = take(R * n.Zp2 * 4);
  p.oEps = take(R * n.Z * 4);
  p.oStd = take(R * n.Z * 4);
  p.oDz = take(R * n.Z * 4);
  const int ub = (2 * n.S > n.H ? 2 * n.S : n.H) * R * 4;
  p.oU = take(ub);
  p.oRch0 = p.oU;
  p.oGd0 = p.oU + R * n.S * 4;
  p.oStart = take(R * 2 * 4);
  p.oRow = take(R * 8);
  p.oMask = take(nmask * R * p.mw * 4);
  p.oPart = take(CVAE_NW * 8 * 4);
  p.total = o;
  return p;
}

// Y = X·Wᵀ over the workgroup's R rows; epi(row0, col, v) receives rows row0..row0+3 of column col.
template <typename T, int R, class Epi>
__device__ __forceinline__ void dense(const T* __restrict__ Xs, int ldx, const T* __restrict__ W,
                                      int Kp, int Np, Epi&& epi) {
  using V = typename Op<T>::V;
  constexpr int EPL = Op<T>::EPL, KC = Op<T>::KC, MT = R / 16, NB = 2, PF = 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = (lane >> 4) * EPL;
  const int NT = Np >> 4, nk = Kp / KC;
  for (int nt0 = wave * NB; nt0 < NT; nt0 += CVAE_NW * NB) {
    f32x4 acc[NB][MT];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[j][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    const T* wp[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) wp[j] = W + (size_t)((nt0 + j) * 16 + r16) * Kp + kq;
    V bq[PF][NB];
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (u < nk) {
#pragma unroll
        for (int j = 0; j < NB; ++j) bq[u][j] = *(const V*)(wp[j] + u * KC);
      }
    for (int kc0 = 0; kc0 < nk; kc0 += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int kc = kc0 + u;
        if (kc < nk) {
          V a[MT];
#pragma unroll
          for (int m = 0; m < MT; ++m) a[m] = *(const V*)(Xs + (m * 16 + r16) * ldx + kc * KC + kq);
#pragma unroll
          for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[j][m] = mfma_chunk(a[m], bq[u][j], acc[j][m]);
          if (kc + PF < nk) {
#pragma unroll
            for (int j = 0; j < NB; ++j) bq[u][j] = *(const V*)(wp[j] + (kc + PF) * KC);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m) epi(m * 16 + (lane >> 4) * 4, (nt0 + j) * 16 + r16, acc[j][m]);
  }
}

template <typename T>
__device__ __forceinline__ void st4(T* p, f32x4 v) {
  if (!CVAE_DIAG_NOSTORE) store4(p, v);
}

__device__ __forceinline__ bool mask_bit(const uint32_t* mk, int mw, int row, int col) {
  return (mk[row * mw + (col >> 5)] >> (col & 31)) & 1u;
}

template <typename T, int R, int MODE>
__global__ __launch_bounds__(CVAE_THREADS) void rowchain_kernel(NetDev net, RowArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const LdsPlan P = lds_plan(net, R, (int)sizeof(T));
  T* Xin = (T*)(smem + P.oXin);
  T* GL = Xin;  // dL/drecon overwrites the input tile in place in the loss epilogue
  T* const P0b = (T*)(smem + P.oP0);
  T* const P1b = (T*)(smem + P.oP1);
  // ping-pong select without a runtime-indexed pointer array (that would live in scratch)
  auto Pb = [&](int i) { return (i & 1) ? P1b : P0b; };
  T* Hc = (T*)(smem + P.oHc);
  T* Q = Hc;    // condition-branch gradient overlays [h_traj ‖ h_c] (dead after fc fwd)
  T* Dec = (T*)(smem + P.oDec);
  T* Cin = (T*)(smem + P.oCin);
  float* MuLv = (float*)(smem + P.oMuLv);
  float* Eps = (float*)(smem + P.oEps);
  float* Std = (float*)(smem + P.oStd);
  float* Dz = (float*)(smem + P.oDz);
  float* Rch0 = (float*)(smem + P.oRch0);
  float* Gd0 = (float*)(smem + P.oGd0);
  float* Dhc2 = (float*)(smem + P.oU);
  float* Start = (float*)(smem + P.oStart);
  int64_t* RowG = (int64_t*)(smem + P.oRow);
  uint32_t* Mask = (uint32_t*)(smem + P.oMask);
  float* Part = (float*)(smem + P.oPart);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = blockIdx.x * R;
  const int nrows = min(R, a.batch - b0);
  const int Bp = net.Bp, Z = net.Z, H = net.H, S = net.S, D = net.D, I = net.I;
  const int mw = P.mw;
  const T* xg = (const T*)a.x;
  constexpr bool TRAIN = MODE == RC_TRAIN;
  const int nmask = 2 + net.n_enc + (net.n_dec - 1);
  const int mC0 = 0, mC1 = 1;
  auto mE = [&](int i) { return 2 + i; };
  auto mD = [&](int i) { return 2 + net.n_enc + i; };

  float s_recon = 0.f, s_kl = 0.f, s_start = 0.f, s_t0 = 0.f, s_relu = 0.f;

  // ---------------------------------------------------------------- phase 0: zero + load
  {
    auto zero = [&](void* p, int bytes) {
      f32x4* q = (f32x4*)p;
      for (int e = tid; e < bytes / 16; e += CVAE_THREADS) q[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    zero(Hc, R * P.shc * (int)sizeof(T));
    zero(Dec, R * P.sdec * (int)sizeof(T));
    zero(Cin, R * P.scin * (int)sizeof(T));
    zero(Mask, rup(nmask * R * mw * 4, 16));
    for (int r = tid; r < R; r += CVAE_THREADS) {
      float s0 = 0.f, s1 = 0.f;
      int64_t g = 0;
      if (r < nrows) {
        g = a.idx ? a.idx[b0 + r] : (int64_t)(b0 + r);
        if (MODE == RC_DECODE || a.x_relative) {
          if (a.start_in) {  // decode(z, h_c) carries no start point
            s0 = a.start_in[(size_t)(b0 + r) * 2 + 0];
            s1 = a.start_in[(size_t)(b0 + r) * 2 + 1];
          }
        } else {
          s0 = to_f(xg[g * I + 1]);   // x[:,0,1:3]  (Training_VAE.py:345)
          s1 = to_f(xg[g * I + 2]);
        }
      }
      Start[r * 2 + 0] = s0;
      Start[r * 2 + 1] = s1;
      RowG[r] = g;
    }
  }
  __syncthreads();
  for (int r = tid; r < nrows; r += CVAE_THREADS) {
    Cin[r * P.scin + 0] = to_t<T>(Start[r * 2 + 0]);
    Cin[r * P.scin + 1] = to_t<T>(Start[r * 2 + 1]);
  }
  if (MODE != RC_DECODE) {
    // relative transform fused into the tile load (Training_VAE.py:347-348)
    using V = typename Op<T>::V;
    constexpr int EPL = Op<T>::EPL, U = 12;
    const bool vec = (I % EPL) == 0 && (((uintptr_t)xg) & 15) == 0;
    if (vec) {
      // 16-B loads, U per thread issued before any is consumed (one memory latency per U·256 vectors)
      const int VPR = I / EPL, NV = R * VPR;
      for (int base = 0; base < NV; base += U * CVAE_THREADS) {
        V buf[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int v = base + u * CVAE_THREADS + tid;
          if (v < NV) {
            const int r = v / VPR, c = v - r * VPR;
            if (r < nrows) buf[u] = *(const V*)(xg + RowG[r] * I + c * EPL);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int v = base + u * CVAE_THREADS + tid;
          if (v < NV) {
            const int r = v / VPR, c = v - r * VPR;
            V o;
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
              float val = 0.f;
              if (r < nrows) {
                val = (float)buf[u][e];
                if (!a.x_relative) {
                  const int d = (c * EPL + e) % D;
                  if (d == 1) val -= Start[r * 2 + 0];
                  else if (d == 2) val -= Start[r * 2 + 1];
                }
              }
              o[e] = to_t<T>(val);
            }
            *(V*)(Xin + r * P.sx + c * EPL) = o;
          }
        }
      }
      if (net.Ip > I) {
        for (int e = tid; e < R * (net.Ip - I); e += CVAE_THREADS) {
          const int r = e / (net.Ip - I), c = I + e % (net.Ip - I);
          Xin[r * P.sx + c] = to_t<T>(0.f);
        }
      }
    } else {
      for (int e = tid; e < R * net.Ip; e += CVAE_THREADS) {
        const int r = e / net.Ip, c = e - r * net.Ip;
        float v = 0.f;
        if (r < nrows && c < I) {
          const int d = c % D;
          v = to_f(xg[RowG[r] * I + c]);
          if (!a.x_relative) {
            if (d == 1) v -= Start[r * 2 + 0];
            else if (d == 2) v -= Start[r * 2 + 1];
          }
        }
        Xin[r * P.sx + c] = to_t<T>(v);
      }
    }
  }
  __syncthreads();
  if (TRAIN && !CVAE_DIAG_NOSTORE) {
    T* xc0 = (T*)net.L[lC0(net)].xT;
    for (int e = tid; e < net.Cp * R; e += CVAE_THREADS) {
      const int c = e / R, r = e - c * R;
      xc0[(size_t)c * Bp + b0 + r] = Cin[r * P.scin + c];
    }
    T* xe0 = (T*)net.L[lE(net, 0)].xT;
    for (int e = tid; e < net.Ip * R; e += CVAE_THREADS) {
      const int c = e / R, r = e - c * R;
      xe0[(size_t)c * Bp + b0 + r] = Xin[r * P.sx + c];
    }
  }

  // Forward ReLU epilogue: LDS dst (+ optional second), arena xT of the consumer, mask bits.
  auto relu_epi = [&](const LayerDev& L, int mi, T* d1, int ld1, int off1, T* d2, int ld2, int off2,
                      T* g1, int goff1, T* g2, int goff2, bool concat) {
    return [&, d1, ld1, off1, d2, ld2, off2, g1, goff1, g2, goff2, concat, mi](int row0, int col, f32x4 v) {
      const float bias = CVAE_DIAG_NOBIAS ? 0.f : L.bias[col];
      f32x4 y;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float t = fmaxf(v[i] + bias, 0.f);
        if (row0 + i >= nrows || col >= L.N) t = 0.f;
        y[i] = t;
        if (t > 0.f) atomicOr(&Mask[(mi * R + row0 + i) * mw + (col >> 5)], 1u << (col & 31));
      }
      if (concat && col >= L.N) return;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        d1[(row0 + i) * ld1 + off1 + col] = to_t<T>(y[i]);
        if (d2) d2[(row0 + i) * ld2 + off2 + col] = to_t<T>(y[i]);
      }
      if (TRAIN) {
        if (g1) st4(g1 + (size_t)(goff1 + col) * Bp + b0 + row0, y);
        if (g2) st4(g2 + (size_t)(goff2 + col) * Bp + b0 + row0, y);
      }
      if (MODE != RC_TRAIN && a.hc_out && mi == mC1 && col < L.N) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (row0 + i < nrows) a.hc_out[(size_t)(b0 + row0 + i) * H + col] = y[i];
      }
    };
  };

  // ---------------------------------------------------------------- condition encoder
  if (MODE == RC_DECODE && a.hc_in) {
    for (int e = tid; e < R * H; e += CVAE_THREADS) {
      const int r = e / H, c = e - r * H;
      Dec[r * P.sdec + Z + c] = to_t<T>(r < nrows ? a.hc_in[(size_t)(b0 + r) * H + c] : 0.f);
    }
    __syncthreads();
  } else {
    const LayerDev& L0 = net.L[lC0(net)];
    dense<T, R>(Cin, P.scin, (const T*)L0.Wf, L0.Kp, L0.Np,
                relu_epi(L0, mC0, Pb(0), P.sp, 0, nullptr, 0, 0, (T*)net.L[lC1(net)].xT, 0, nullptr, 0, false));
    __syncthreads();
    const LayerDev& L1 = net.L[lC1(net)];
    dense<T, R>(Pb(0), P.sp, (const T*)L1.Wf, L1.Kp, L1.Np,
                relu_epi(L1, mC1, Hc, P.shc, H, Dec, P.sdec, Z, (T*)net.L[lFC(net)].xT, H,
                         (T*)net.L[lD(net, 0)].xT, Z, true));
    __syncthreads();
  }

  if (MODE != RC_DECODE) {
    // ---------------------------------------------------------------- encoder
    const T* in = Xin;
    int ldin = P.sx;
    for (int i = 0; i < net.n_enc; ++i) {
      const LayerDev& L = net.L[lE(net, i)];
      const bool last = i == net.n_enc - 1;
      if (last)
        dense<T, R>(in, ldin, (const T*)L.Wf, L.Kp, L.Np,
                    relu_epi(L, mE(i), Hc, P.shc, 0, nullptr, 0, 0, (T*)net.L[lFC(net)].xT, 0, nullptr, 0, true));
      else
        dense<T, R>(in, ldin, (const T*)L.Wf, L.Kp, L.Np,
                    relu_epi(L, mE(i), Pb(i & 1), P.sp, 0, nullptr, 0, 0, (T*)net.L[lE(net, i + 1)].xT, 0,
                             nullptr, 0, false));
      __syncthreads();
      in = Pb(i & 1);
      ldin = P.sp;
    }
    // ---------------------------------------------------------------- fc_mu ‖ fc_logvar
    {
      const LayerDev& L = net.L[lFC(net)];
      dense<T, R>(Hc, P.shc, (const T*)L.Wf, L.Kp, L.Np, [&](int row0, int col, f32x4 v) {
        const float bias = CVAE_DIAG_NOBIAS ? 0.f : L.bias[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = row0 + i;
          const float t = (row < nrows && col < L.N) ? v[i] + bias : 0.f;
          MuLv[row * net.Zp2 + col] = t;
          if (MODE == RC_FWD && row < nrows && col < L.N) {
            if (col < Z) { if (a.mu_out) a.mu_out[(size_t)(b0 + row) * Z + col] = t; }
            else if (a.lv_out) a.lv_out[(size_t)(b0 + row) * Z + col - Z] = t;
          }
        }
      });
      __syncthreads();
    }
    // ---------------------------------------------------------------- reparameterize (:199-206) + KL terms (:243)
    {
      T* xd0 = (T*)net.L[lD(net, 0)].xT;
      for (int e = tid; e < R * Z; e += CVAE_THREADS) {
        const int r = e / Z, j = e - r * Z;
        float z = 0.f, ep = 0.f, sd = 0.f;
        if (r < nrows) {
          const float mu = MuLv[r * net.Zp2 + j], lv = MuLv[r * net.Zp2 + Z + j];
          sd = expf(0.5f * lv);
          ep = a.eps ? a.eps[(size_t)(b0 + r) * Z + j] : philox_normal(a.seed, a.offset, (uint32_t)(b0 + r), (uint32_t)j);
          z = mu + ep * sd;
          s_kl += 1.f + lv - mu * mu - expf(lv);
        }
        Eps[r * Z + j] = ep;
        Std[r * Z + j] = sd;
        Dec[r * P.sdec + j] = to_t<T>(z);
        if (TRAIN && !CVAE_DIAG_NOSTORE) xd0[(size_t)j * Bp + b0 + r] = to_t<T>(z);
      }
      __syncthreads();
    }
  } else {
    if (!a.z_in) return;  // condition encoder only (cvae_condition)
    for (int e = tid; e < R * Z; e += CVAE_THREADS) {
      const int r = e / Z, j = e - r * Z;
      Dec[r * P.sdec + j] = to_t<T>(r < nrows ? a.z_in[(size_t)(b0 + r) * Z + j] : 0.f);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- decoder
  const int nd = net.n_dec;
  const T* din = Dec;
  int lddin = P.sdec;
  for (int i = 0; i < nd - 1; ++i) {
    const LayerDev& L = net.L[lD(net, i)];
    dense<T, R>(din, lddin, (const T*)L.Wf, L.Kp, L.Np,
                relu_epi(L, mD(i), Pb(i & 1), P.sp, 0, nullptr, 0, 0, (T*)net.L[lD(net, i + 1)].xT, 0,
                         nullptr, 0, false));
    __syncthreads();
    din = Pb(i & 1);
    lddin = P.sp;
  }
  const LayerDev& LL = net.L[lD(net, nd - 1)];
  const float Bf = (float)a.batch;
  const float inv_BSD = 1.f / (Bf * (float)(S * D));
  const float inv_2B = 1.f / (2.f * Bf);
  const float inv_B = 1.f / Bf;
  const float inv_BS1 = S > 1 ? 1.f / (Bf * (float)(S - 1)) : 0.f;
  const float inv_BZ = 1.f / (Bf * (float)Z);
  if (!TRAIN) {
    dense<T, R>(din, lddin, (const T*)LL.Wf, LL.Kp, LL.Np, [&](int row0, int col, f32x4 v) {
      if (col >= I || !a.recon_out) return;
      const float bias = CVAE_DIAG_NOBIAS ? 0.f : LL.bias[col];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (row0 + i < nrows) a.recon_out[(size_t)(b0 + row0 + i) * I + col] = v[i] + bias;
    });
    return;
  }
  // loss epilogue: recon r = acc + bias stays fp32; dL/dr into GL (LDS) and gT(D_last)
  {
    T* gl = (T*)LL.gT;
    const bool use_start = a.w_start > 0.f, use_time = a.w_time > 0.f;  // :247, :256
    dense<T, R>(din, lddin, (const T*)LL.Wf, LL.Kp, LL.Np, [&](int row0, int col, f32x4 v) {
      const float bias = CVAE_DIAG_NOBIAS ? 0.f : LL.bias[col];
      const int s = col / D, d = col - s * D;
      f32x4 g;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = row0 + i;
        float gi = 0.f;
        if (row < nrows && col < I) {
          const float r = v[i] + bias;
          // target x_rel from the resident input tile; GL overwrites it in place below
          // (same lane, same element), so no other reader is affected
          const float xr = to_f(Xin[row * P.sx + col]);
          const float diff = r - xr;
          s_recon += diff * diff;
          gi = a.w_recon * 2.f * diff * inv_BSD;
          if (s == 0 && (d == 1 || d == 2) && use_start) {
            s_start += diff * diff;
            gi += a.w_start * 2.f * diff * inv_2B;
          }
          if (d == 0) {
            Rch0[row * S + s] = r;
            if (s == 0 && use_time) {
              s_t0 += r * r;
              gi += a.w_time * 2.f * r * inv_B;
            }
            Gd0[row * S + s] = gi;
          }
        }
        g[i] = gi;
      }
      if (d == 0 && col < I) return;  // time-channel gradient finished after the neighbours exist
#pragma unroll
      for (int i = 0; i < 4; ++i) GL[(row0 + i) * P.sx + col] = to_t<T>(g[i]);
      st4(gl + (size_t)col * Bp + b0 + row0, g);
    });
    __syncthreads();
    // time-monotonicity term: relu(r_s - r_{s+1}) (:261-262), ReLU'(0) = 0
    for (int e = tid; e < R * S; e += CVAE_THREADS) {
      const int r = e / S, s = e - r * S;
      float g = 0.f;
      if (r < nrows) {
        g = Gd0[r * S + s];
        if (use_time) {
          if (s < S - 1) {
            const float u = Rch0[r * S + s] - Rch0[r * S + s + 1];
            if (u > 0.f) { g += a.w_time * inv_BS1; s_relu += u; }
          }
          if (s > 0) {
            const float u = Rch0[r * S + s - 1] - Rch0[r * S + s];
            if (u > 0.f) g -= a.w_time * inv_BS1;
          }
        }
      }
      GL[r * P.sx + s * D] = to_t<T>(g);
      if (!CVAE_DIAG_NOSTORE) gl[(size_t)(s * D) * Bp + b0 + r] = to_t<T>(g);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- backward
  // dX = G·W with W from the transposed copy Wb[Kp][Np]; mask with the producer's ReLU bits.
  auto bwd_epi = [&](int mi, T* dst, int ld, T* gdst) {
    return [&, mi, dst, ld, gdst](int row0, int col, f32x4 v) {
      f32x4 g;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        g[i] = mask_bit(Mask + mi * R * mw, mw, row0 + i, col) ? v[i] : 0.f;
      if (dst) {
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[(row0 + i) * ld + col] = to_t<T>(g[i]);
      }
      st4(gdst + (size_t)col * Bp + b0 + row0, g);
    };
  };
  const T* gin = GL;
  int ldg = P.sx;
  int pp = 0;
  for (int i = nd - 1; i >= 1; --i) {
    const LayerDev& L = net.L[lD(net, i)];
    dense<T, R>(gin, ldg, (const T*)L.Wb, L.Np, L.Kp,
                bwd_epi(mD(i - 1), Pb(pp), P.sp, (T*)net.L[lD(net, i - 1)].gT));
    __syncthreads();
    gin = Pb(pp);
    ldg = P.sp;
    pp ^= 1;
  }
  {  // decoder L0 backward splits into dz and the decoder's share of dh_c
    const LayerDev& L = net.L[lD(net, 0)];
    dense<T, R>(gin, ldg, (const T*)L.Wb, L.Np, L.Kp, [&](int row0, int col, f32x4 v) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (col < Z) Dz[(row0 + i) * Z + col] = v[i];
        else if (col < Z + H) Dhc2[(row0 + i) * H + col - Z] = v[i];
      }
    });
    __syncthreads();
  }
  {  // reparameterisation + KL backward → G_fc = [dmu ‖ dlogvar]
    const LayerDev& L = net.L[lFC(net)];
    T* gfc = (T*)L.gT;
    T* P0 = Pb(0);
    for (int e = tid; e < R * net.Zp2; e += CVAE_THREADS) {
      const int r = e / net.Zp2, c = e - r * net.Zp2;
      float g = 0.f;
      if (r < nrows && c < 2 * Z) {
        const int j = c < Z ? c : c - Z;
        const float dz = Dz[r * Z + j];
        if (c < Z) {
          g = a.w_kld * MuLv[r * net.Zp2 + j] * inv_BZ + dz;
        } else {
          const float lv = MuLv[r * net.Zp2 + Z + j];
          g = a.w_kld * 0.5f * (expf(lv) - 1.f) * inv_BZ + dz * Eps[r * Z + j] * 0.5f * Std[r * Z + j];
        }
      }
      P0[r * P.sp + c] = to_t<T>(g);
      if (!CVAE_DIAG_NOSTORE) gfc[(size_t)c * Bp + b0 + r] = to_t<T>(g);
    }
    // pads of the two gradient targets of the fc backward must read as zero
    if (net.Hp > H) {
      for (int e = tid; e < R * (net.Hp - H); e += CVAE_THREADS) {
        const int r = e / (net.Hp - H), c = H + e % (net.Hp - H);
        Pb(1)[r * P.sp + c] = to_t<T>(0.f);
        Q[r * P.shc + c] = to_t<T>(0.f);
      }
    }
    __syncthreads();
    // fc backward: dh = G_fc·W_fc → [dh_traj ‖ dh_c(fc share)]
    T* ge = (T*)net.L[lE(net, net.n_enc - 1)].gT;
    T* gc1 = (T*)net.L[lC1(net)].gT;
    const uint32_t* mkE = Mask + mE(net.n_enc - 1) * R * mw;
    const uint32_t* mkC = Mask + mC1 * R * mw;
    dense<T, R>(P0, P.sp, (const T*)L.Wb, L.Np, L.Kp, [&](int row0, int col, f32x4 v) {
      f32x4 g;
      if (col < H) {
#pragma unroll
        for (int i = 0; i < 4; ++i) g[i] = mask_bit(mkE, mw, row0 + i, col) ? v[i] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) Pb(1)[(row0 + i) * P.sp + col] = to_t<T>(g[i]);
        st4(ge + (size_t)col * Bp + b0 + row0, g);
      } else if (col < 2 * H) {
        const int c = col - H;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          g[i] = mask_bit(mkC, mw, row0 + i, c) ? v[i] + Dhc2[(row0 + i) * H + c] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) Q[(row0 + i) * P.shc + c] = to_t<T>(g[i]);
        st4(gc1 + (size_t)c * Bp + b0 + row0, g);
      }
    });
    __syncthreads();
  }
  {  // encoder backward (G of E0 is the last one needed: the input has no grad)
    const T* g = Pb(1);
    int p = 0;
    for (int i = net.n_enc - 1; i >= 1; --i) {
      const LayerDev& L = net.L[lE(net, i)];
      dense<T, R>(g, P.sp, (const T*)L.Wb, L.Np, L.Kp,
                  bwd_epi(mE(i - 1), i > 1 ? Pb(p) : nullptr, P.sp, (T*)net.L[lE(net, i - 1)].gT));
      __syncthreads();
      g = Pb(p);
      p ^= 1;
    }
    // condition encoder L2 backward → G of condition L1
    const LayerDev& L = net.L[lC1(net)];
    dense<T, R>(Q, P.shc, (const T*)L.Wb, L.Np, L.Kp, bwd_epi(mC0, nullptr, 0, (T*)net.L[lC0(net)].gT));
  }

  // ---------------------------------------------------------------- loss partial sums (deterministic order)
  s_recon = wave_sum(s_recon);
  s_kl = wave_sum(s_kl);
  s_start = wave_sum(s_start);
  s_t0 = wave_sum(s_t0);
  s_relu = wave_sum(s_relu);
  if (lane == 0) {
    Part[wave * 8 + 0] = s_recon;
    Part[wave * 8 + 1] = s_kl;
    Part[wave * 8 + 2] = s_start;
    Part[wave * 8 + 3] = s_t0;
    Part[wave * 8 + 4] = s_relu;
  }
  __syncthreads();
  if (tid < 5) {
    float s = 0.f;
    for (int w = 0; w < CVAE_NW; ++w) s += Part[w * 8 + tid];
    a.partials[blockIdx.x * 8 + tid] = s;
  }
}
