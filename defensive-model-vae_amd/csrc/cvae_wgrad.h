// cvae_wgrad.h — weight/bias gradients (a batch reduction) and the Adam update.
//
// wgrad_kernel: one workgroup per 32×32 tile of one layer's padded weight
// matrix.  dW_l[o][i] = Σ_b gT(l)[o][b] · xT(l)[i][b]  (dW = Gᵀ·X,
// K = batch), both operands batch-contiguous in the activation arena, MFMA
// 16x16x32 bf16 (or 4×16x16x4 f32) with the K range split over the 4 waves
// and combined through LDS in a fixed order (deterministic).  Tiles with
// i0 == 0 also reduce the bias gradient db = Σ_b G from the G fragments the
// MFMA loop already holds (no second pass over the rows).
//
// The epilogue either writes the fp32 gradient into the flat state_dict-ordered
// buffer (data-parallel path: all-reduce comes next) or applies torch's Adam
// (torch/optim/adam.py _single_tensor_adam, replacing optimizer.step() at
// Training_VAE.py:363) in place and refreshes the padded operand copies
// Wf/Wb/bias that the row-chain kernel reads — the gradient never round-trips
// through HBM.  param_kernel does the same update from a gradient buffer
// (after the all-reduce) or just repacks the copies (PACK).
//
// Epilogue shape: a thread owns 4 consecutive inputs (o, i..i+3) of one output row and issues
// all its p/m/v loads before any store; the new weights go through an LDS image of the tile so
// that each operand copy is written as whole 16-B MFMA fragments (1 KB per wave instruction)
// instead of 2-B element stores scattered over the fragment layout.
#pragma once
#include <type_traits>
#include "cvae_device.h"
#include "cvae_peer.h"

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
    if (threadIdx.x == 0 && g_wstamps) g_wstamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define WSTAMP(k) do { } while (0)
#endif
#ifndef CVAE_DIAG_WSTAMP_ENTRY
#define CVAE_DIAG_WSTAMP_ENTRY 0  // diagnostic builds: stamp 0 at kernel entry, before the tile decode
#endif

struct AdamArgs {
  float* params;      // flat fp32 master (state_dict order)
  float* m;
  float* v;
  float* grads;       // PM_GRAD: output; param_kernel PM_ADAM: input
  float grad_scale;
  float lr_neg_step;  // -lr / (1 - beta1^t)        (host path; device path: adam_resolve)
  float bc2_sqrt;     // sqrt(1 - beta2^t)
  float beta1_w;      // 1 - beta1  (lerp weight)
  float beta2;
  float one_m_beta2;
  float eps;
  int pad_;
  const uint64_t* ctr;  // device step counters (cvae.h): t = ctr[1]; NULL = the two scalars above
  double lr, beta1d, beta2d;
};

// device-counter path: the step's two scalars are precomputed once per step (by the row chain that
// begins the step, adam_precompute) into ctr[2] as two fp32 — a kernel loads 8 bytes instead of
// doing double pow in every block.  Issued first (vmcnt retires in order).
__device__ __forceinline__ adam_f32x2 adam_step_load(const AdamArgs& a) {
  return a.ctr ? gld<adam_f32x2>(a.ctr + 2) : adam_f32x2{0.f, 0.f};
}
__device__ __forceinline__ void adam_resolve(AdamArgs& a, adam_f32x2 sc) {
  if (a.ctr) {
    a.lr_neg_step = sc[0];
    a.bc2_sqrt = sc[1];
  }
}
struct LossArgs {
  const float* partials;  // [ntiles][8]
  int ntiles;
  int batch;
  float w_recon, w_kld, w_start, w_time;
  float* loss_out;        // [5] nullable
  double* loss_accum;     // [5] nullable, += (double)loss * batch (Training_VAE.py:366-370 in doubles)
  uint64_t* ctr;          // device step counters: the loss finisher advances ctr[0] (Philox offset)
};

#ifndef CVAE_DIAG_NOADAM
#define CVAE_DIAG_NOADAM 0  // timing only: the update is p − lr·g (no moments)
#endif
// One element of torch's Adam, in its op order; m and v are updated in place.
// No FMA contraction inside (hipcc contracts across statements by default): every kernel that applies
// Adam — the fused dW ⊕ Adam epilogues, param_kernel, the peer exchange's owners, the sharded flat Adam
// (cvae_adam_flat) — rounds each torch op separately, so they agree bit for bit whatever code
// surrounds the inlined call.
#ifndef CVAE_ADAM_CONTRACT
#define CVAE_ADAM_CONTRACT 0  // diagnostic builds only: hipcc's default contraction (the A/B of its cost)
#endif
__device__ __forceinline__ float adam_math(float p, float g, float& m, float& v, const AdamArgs& a) {
#if !CVAE_ADAM_CONTRACT
#pragma clang fp contract(off)
#endif
  if (CVAE_DIAG_NOADAM) return p + a.lr_neg_step * g;
  // exp_avg.lerp_(grad, 1 - beta1): weight < 0.5 branch of at::lerp
  m = a.beta1_w < 0.5f ? m + a.beta1_w * (g - m) : g - (g - m) * (1.f - a.beta1_w);
  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
  v = v * a.beta2;
  v = v + a.one_m_beta2 * g * g;
  // denom = exp_avg_sq.sqrt() / bias_correction2_sqrt + eps;  param.addcdiv_(exp_avg, denom, -step_size)
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  return p + a.lr_neg_step * m / denom;
}

// LDS image of one 32×32 tile: fp32 rows padded to 36 floats (16-B aligned rows)
constexpr int WT_LD = 36;

// EPT consecutive fp32 values (the per-thread share of a tile's epilogue)
template <int EPT> struct VecF;
template <> struct VecF<2> { typedef float T __attribute__((ext_vector_type(2))); };
template <> struct VecF<4> { typedef f32x4 T; };

// The fp32 master state of weights (o, i..i+EPT-1) of layer L (padded coordinates), loaded before
// the gradient exists (it does not depend on it) so the epilogue is arithmetic and stores only.
template <int EPT>
struct PreN {
  float p[EPT], m[EPT], v[EPT];
  int64_t base;
  int64_t stride;  // flat distance of consecutive inputs i (1; N for a [K][N]-stored table)
  int nv;    // valid elements (0: padding)
  bool vec;  // whole aligned vector runs (layer-uniform)
};
template <int MODE, int EPT>
__device__ __forceinline__ PreN<EPT> loadn(const LayerDev& L, int o, int i, const AdamArgs& a) {
  using V = typename VecF<EPT>::T;
  PreN<EPT> s;
  s.nv = 0;
  s.base = 0;
#pragma unroll
  for (int c = 0; c < EPT; ++c) s.p[c] = s.m[c] = s.v[c] = 0.f;
  // wave-uniform: every run of the layer is an aligned EPT-vector (K % EPT == 0, segment offsets
  // % EPT == 0).  The choice must not be per lane: divergent scalar and vector paths share
  // destination registers, and the vector path then waits (vmcnt(0)) for every load in flight
  s.vec = !L.wt && (L.K % EPT) == 0 && ((L.pw[0] | L.pw[1]) % EPT) == 0;
  s.stride = L.wt ? L.N : 1;
  if (o >= L.N || i >= L.K) return s;
  const int seg = (L.nseg == 2 && o >= L.seg_rows0) ? 1 : 0;
  s.base = L.wt ? L.pw[0] + (int64_t)i * L.N + o : L.pw[seg] + (int64_t)(seg ? o - L.seg_rows0 : o) * L.K + i;
  s.nv = min(EPT, L.K - i);
  if (MODE == PM_GRAD) return s;
  if (s.vec) {
    const V pv = *(const V*)(a.params + s.base);
#pragma unroll
    for (int c = 0; c < EPT; ++c) s.p[c] = pv[c];
    if (MODE == PM_ADAM) {
      const V mv = *(const V*)(a.m + s.base), vv = *(const V*)(a.v + s.base);
#pragma unroll
      for (int c = 0; c < EPT; ++c) {
        s.m[c] = mv[c];
        s.v[c] = vv[c];
      }
    }
    return s;
  }
#pragma unroll
  for (int c = 0; c < EPT; ++c) {
    if (c < s.nv) {
      s.p[c] = a.params[s.base + c * s.stride];
      if (MODE == PM_ADAM) {
        s.m[c] = a.m[s.base + c * s.stride];
        s.v[c] = a.v[s.base + c * s.stride];
      }
    }
  }
  return s;
}
// write the gradient (GRAD), apply Adam (ADAM) or keep (PACK); returns the values for the operand
// copies (0 in the padding)
template <int MODE, int EPT>
__device__ __forceinline__ typename VecF<EPT>::T applyn(PreN<EPT> s, typename VecF<EPT>::T g,
                                                        const AdamArgs& a) {
  using V = typename VecF<EPT>::T;
  V w = {};
  if (MODE == PM_GRAD) {
#pragma unroll
    for (int c = 0; c < EPT; ++c)
      if (c < s.nv) a.grads[s.base + c * s.stride] = g[c];
    return w;
  }
  if (MODE == PM_ADAM) {
#pragma unroll
    for (int c = 0; c < EPT; ++c) s.p[c] = adam_math(s.p[c], g[c], s.m[c], s.v[c], a);
    if (s.vec) {
      if (s.nv == EPT) {
        V pv, mv, vv;
#pragma unroll
        for (int c = 0; c < EPT; ++c) {
          pv[c] = s.p[c];
          mv[c] = s.m[c];
          vv[c] = s.v[c];
        }
        st_wt(a.params, (size_t)s.base * 4, pv);
        st_wt(a.m, (size_t)s.base * 4, mv);
        st_wt(a.v, (size_t)s.base * 4, vv);
      }
    } else {
#pragma unroll
      for (int c = 0; c < EPT; ++c) {
        if (c < s.nv) {
          a.params[s.base + c * s.stride] = s.p[c];
          a.m[s.base + c * s.stride] = s.m[c];
          a.v[s.base + c * s.stride] = s.v[c];
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < EPT; ++c) w[c] = c < s.nv ? s.p[c] : 0.f;
  return w;
}

// the master state of bias o (padded coordinate) of layer L, loaded early like PreN
struct PreB {
  float p, m, v;
  int64_t idx;  // -1: padding
};
template <int MODE>
__device__ __forceinline__ PreB loadb(const LayerDev& L, int o, const AdamArgs& a) {
  PreB b{0.f, 0.f, 0.f, -1};
  if (o >= L.N || !L.has_bias) return b;
  const int seg = (L.nseg == 2 && o >= L.seg_rows0) ? 1 : 0;
  b.idx = L.pb[seg] + (seg ? o - L.seg_rows0 : o);
  if (MODE == PM_GRAD) return b;
  b.p = a.params[b.idx];
  if (MODE == PM_ADAM) {
    b.m = a.m[b.idx];
    b.v = a.v[b.idx];
  }
  return b;
}
// returns the padded bias value written to L.bias (the peer exchange broadcasts it)
template <int MODE>
__device__ __forceinline__ float apply_bias(const LayerDev& L, int o, PreB b, float g, const AdamArgs& a) {
  if (o >= L.Np) return 0.f;
  float w = 0.f;
  if (b.idx >= 0) {
    if (MODE == PM_GRAD) { a.grads[b.idx] = g; return 0.f; }
    w = b.p;
    if (MODE == PM_ADAM) {
      w = adam_math(w, g, b.m, b.v, a);
      st_wt(a.params, (size_t)b.idx * 4, w);
      st_wt(a.m, (size_t)b.idx * 4, b.m);
      st_wt(a.v, (size_t)b.idx * 4, b.v);
    }
  } else if (MODE == PM_GRAD) {
    return 0.f;
  }
  if (CVAE_DIAG_NOWPACK && MODE == PM_ADAM) return w;
  st_wt(L.bias, (size_t)o * 4, w);
  return w;
}

// Both operand copies of one 32×32 tile from its LDS image, as whole MFMA fragments.  Fragment
// (n-tile t, chunk kc) lane ln holds elements (16t + (ln & 15), KC·kc + frag_k(ln >> 4, e)) at
// ((t·Kp/KC + kc)·64 + ln)·EPL (frag_off), so a tile is 2 n-tiles × 32/KC chunks of contiguous
// 1-KB blocks per copy.
// SYS (the peer exchange's broadcast into another rank's arena): every piece a system-scope
// write-through store (relaxed system atomics, 8 B each), so a drain, not a cache write-back, puts
// it in that rank's memory
template <bool SYS, typename V>
__device__ __forceinline__ void op_st(void* base, size_t byte_off, V v) {
  if constexpr (SYS) {
    static_assert(sizeof(V) % 8 == 0, "8- or 16-B fragments");
    typedef unsigned long long u64v __attribute__((ext_vector_type(sizeof(V) / 8)));
    const u64v w = __builtin_bit_cast(u64v, v);
#pragma unroll
    for (int c = 0; c < (int)(sizeof(V) / 8); ++c)
      __hip_atomic_store((uint64_t*)((char*)base + byte_off) + c, (uint64_t)w[c], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    st_wt(base, byte_off, v);
  }
}

template <typename T, int NTHR, int LD = WT_LD, bool SYS = false>
__device__ __forceinline__ void store_operands(const LayerDev& L, int o0, int i0, const float* wt) {
  using V = typename Op<T>::V;
  constexpr int EPL = Op<T>::EPL, KC = Op<T>::KC, CPT = 32 / KC;
  constexpr int PER_COPY = 2 * CPT * 64;
#pragma unroll
  for (int j0 = 0; j0 < 2 * PER_COPY; j0 += NTHR) {
    const int j = j0 + (int)threadIdx.x;
    if (NTHR > 2 * PER_COPY && j >= 2 * PER_COPY) break;
    const bool wb = j >= PER_COPY;  // wave-uniform: PER_COPY is a multiple of 64
    const int jj = wb ? j - PER_COPY : j;
    const int blk = jj >> 6, ln = jj & 63;
    const int bt = blk / CPT, bk = blk - bt * CPT;
    const int nl = bt * 16 + (ln & 15), kl = bk * KC, q = ln >> 4;  // lane (nl, q) of chunk kl
    V val;
    if (wb) {  // Wb = Wᵀ: rows = inputs i, K = outputs o
#pragma unroll
      for (int e = 0; e < EPL; ++e) val[e] = to_t<T>(wt[(kl + frag_k<T>(q, e)) * LD + nl]);
      op_st<SYS>(L.Wb, ((size_t)(((i0 >> 4) + bt) * (L.Np / KC) + (o0 + kl) / KC) * 64 + ln) * EPL * sizeof(T), val);
      if constexpr (EPL == 8 && !SYS) {
        if (L.f8b) {  // the wide chain's e4m3 dX operand: e4m3(s·Wᵀ) in K-pair fragments (K = the outputs)
          const float sc = f8_header(L.Wf)->s;
          float f[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = wt[(kl + frag_k<T>(q, e)) * LD + nl] * sc;
          gst<long>((long*)((char*)L.Wb8 + f8_wf_off(i0 + bt * 16, (o0 + kl) / 32, L.Np) + (size_t)ln * 16), f8x8(f));
        }
      }
    } else if (EPL == 8 && L.f8) {  // CVAE_FP8: e4m3(s·W), 8 B per lane into its K-pair fragment
      const float sc = f8_header(L.Wf)->s;
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; e += 4) {
        const f32x4 v4 = *(const f32x4*)(wt + nl * LD + kl + frag_k<T>(q, e));
#pragma unroll
        for (int c = 0; c < 4; ++c) f[e + c] = v4[c] * sc;
      }
      const size_t off = f8_wf_off(o0 + bt * 16, (i0 + kl) / 32, L.Kp) + (size_t)ln * 16;
      if constexpr (SYS) op_st<true>(L.Wf, off, f8x8(f));
      else gst<long>((long*)((char*)L.Wf + off), f8x8(f));
    } else {
#pragma unroll
      for (int e = 0; e < EPL; e += 4) {  // 4 consecutive K positions per half-fragment
        const f32x4 v4 = *(const f32x4*)(wt + nl * LD + kl + frag_k<T>(q, e));
#pragma unroll
        for (int c = 0; c < 4; ++c) val[e + c] = to_t<T>(v4[c]);
      }
      op_st<SYS>(L.Wf, ((size_t)(((o0 >> 4) + bt) * (L.Kp / KC) + (i0 + kl) / KC) * 64 + ln) * EPL * sizeof(T), val);
    }
  }
}

// Shared by wgrad_kernel and param_kernel.  The tile is 32 outputs × 32·NI inputs; thread
// (o = tid/TPR, i = EPT·(tid%TPR)), TPR = 32·NI/EPT, owns the gradient g of weights
// (o0+o, i0+i..+EPT-1) (state st from loadn); threads < 32 own bias o0+tid (tiles with i0 == 0).
// wt: an LDS tile image (32 rows of 32·NI + 4 floats) the caller no longer needs.  Every thread of
// the block calls it (barrier inside).
// returns (threads < 32 of a tile with i0 == 0) the new padded bias value, else 0
template <typename T, int MODE, int NTHR, int EPT, int NI = 1>
__device__ __forceinline__ float tile_epilogue(const LayerDev& L, int o0, int i0, const PreN<EPT>& st, const PreB& sb,
                                              typename VecF<EPT>::T g, float db, const AdamArgs& aa, float* wt) {
  using V = typename VecF<EPT>::T;
  constexpr int TW = 32 * NI, LD = TW + 4, TPR = TW / EPT;  // tile width, image row stride, threads per row
  const int tid = threadIdx.x, o = tid / TPR, iv = (tid % TPR) * EPT;
  V w = {};
  if (tid < 32 * TPR) w = applyn<MODE, EPT>(st, g, aa);
  WSTAMP(4);
  float nb = 0.f;
  if (i0 == 0 && tid < 32) nb = apply_bias<MODE>(L, o0 + tid, sb, db, aa);
  if (MODE == PM_GRAD || (CVAE_DIAG_NOWPACK && MODE == PM_ADAM)) return nb;
  if (tid < 32 * TPR) *(V*)(wt + o * LD + iv) = w;
  __syncthreads();
  WSTAMP(5);
#pragma unroll
  for (int s = 0; s < NI; ++s) store_operands<T, NTHR, LD>(L, o0, i0 + 32 * s, wt + 32 * s);
  WSTAMP(6);
  return nb;
}

// peer exchange (cvae_peer.h): after the owner's tile_epilogue, the same new operand copies (the
// LDS image wt) and bias into every other rank's arena, released at system scope, then one arrival
// on each of their done counters
template <typename T, int NTHR>
__device__ __forceinline__ void px_broadcast(const PeerArgs& p, const LayerDev& L, int o0, int i0, const float* wt,
                                             float nb) {
  const int tid = threadIdx.x;
  for (int r = 0; r < p.world; ++r) {
    if (r == p.rank) continue;
    const ptrdiff_t d = p.arena[r] - p.arena[p.rank];
    LayerDev Lr = L;
    Lr.Wf = (char*)L.Wf + d;
    Lr.Wb = (char*)L.Wb + d;
    store_operands<T, NTHR, WT_LD, (bool)CVAE_PX_SC>(Lr, o0, i0, wt);
    if (i0 == 0 && tid < 32 && o0 + tid < L.Np) {
      float* const bd = (float*)((char*)(L.bias + o0 + tid) + d);
      if (CVAE_PX_SC) __hip_atomic_store((unsigned*)bd, __builtin_bit_cast(unsigned, nb), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
      else *bd = nb;
    }
  }
  if (CVAE_PX_SC) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every piece in the peers' memory first
  else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (tid < p.world && tid != p.rank)
    __hip_atomic_fetch_add(px_done(p, p.mbox[tid]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// called by one whole wave: lane-strided partial sums, then a fixed-order butterfly (deterministic).
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
    if (l.loss_accum) l.loss_accum[k] += (double)v[k] * (double)l.batch;
  }
  // the step's row chain has read the Philox offset (previous launch): advance it for the next step
  if (l.ctr) l.ctr[0] = l.ctr[0] + 1;
}

// 8 waves per tile: the batch (K) is cut into 8 wave slices whose loads are all in flight at once
constexpr int WG_NW = 8, WG_THREADS = 64 * WG_NW;

// LDS of one dW workgroup for tiles up to 32·NI inputs wide
template <int NI>
struct WgradLds {
  float red[WG_NW * 32 * (32 * NI + 4)];  // per-wave partial tiles, then the new weights' image
  float dbp[WG_NW * 32];                  // per-wave bias partials
};

// Split-K over the batch (large batches): split sk.s of sk.S computes the tile's partial dW/db over
// its K range, writes it (fp32, write-through) to sk.ws, and adds to the tile's ticket; the block
// whose add returns S-1 sums the S partials in split order (deterministic, independent of arrival
// order) and runs the epilogue, then zeroes the ticket for the next launch (MI355X_MICROARCH.md,
// inter-workgroup hand-off: sc1 stores drained before one lane's agent-scope add; the last adder
// reads with sc1 loads after a workgroup barrier).  S = 1: the whole batch in one block.
struct SplitK {
  int S, s;
  float* ws;          // [tile][S][pw] fp32 partials (dW then db)
  unsigned* tickets;  // [tile], zero between launches
  int tile;
  int pw;             // floats per partial (0: 32·TW + 32 of the tile)
};

// ---- MX dW (CVAE_FP8_DW=mx: the wide fp8 form's 32 × 64 tiles, batch a multiple of 128).  One
// 128-row chunk of the batch (K) per block-scaled MFMA; every 32 consecutive rows of one feature are
// one MX block, converted by the consumer — the chain's 16-row workgroups cannot form them (DESIGN
// §4.5).  Lane r + 16j loads, as quarter h, the 8 rows 32·(2(h >> 1) + (j >> 1)) + 8·(2(h & 1) + (j & 1))
// of its feature, so the instruction's block b (quarters 2(b >> 1), +1 of the lanes j = 2(b & 1), +1)
// is rows 32b..32b+31 (oracle/cvae_np.py mx_dw; tests/test_mx_oracle.py checks the two agree).
// mx_block converts a lane's quarters and returns its lane pair's two block exponents; the scale
// lane r + 16j hands the instruction (block j: half j >> 1 of pair j & 1) comes from lane
// r + 32(j & 1) by one ds_bpermute.  The X n-tiles stream one ahead of their conversion (the
// operand registers of two workgroups per CU).
__device__ __forceinline__ size_t mx_row(int h, int j) {
  return (size_t)(32 * (2 * (h >> 1) + (j >> 1)) + 8 * (2 * (h & 1) + (j & 1)));
}
__device__ __forceinline__ int mx_scale(unsigned p, int lane) {
  const int j = lane >> 4;
  const unsigned pp = (unsigned)__builtin_amdgcn_ds_bpermute(((lane & 15) + 32 * (j & 1)) << 2, (int)p);
  return 127 - mx_k((int)(pp >> (16 * (j >> 1))) & 0xffff);
}
// G, X: the layer's arena matrices (block-uniform: buffer resources, no 64-bit lane addresses);
// fo, fi: this lane's first output / input feature (o0 + r, i0 + r); ct: the chunk's first row
template <int NX>
__device__ __forceinline__ void mx_dw_chunk(const __bf16* G, const __bf16* X, int fo, int fi, int ct, int Kg, int Kx,
                                            f32x4 (&acc)[2][NX], float (&gs)[2], bool bias_tile) {
  const int lane = threadIdx.x & 63, j = lane >> 4;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, 0x7fffffff, 0x00020000);
  auto bo = [](int f, int row, int Kf) { return (((row >> 4) * Kf + f) * 16 + (row & 15)) * 2; };  // aoff, bytes
  auto ld = [](__amdgpu_buffer_rsrc_t rs, int off) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  };
  int r[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) r[h] = ct + (int)mx_row(h, j);
  auto ldx = [&](bf16x8 (&d)[4], int n) {
#pragma unroll
    for (int h = 0; h < 4; ++h) d[h] = ld(rx, bo(fi + 16 * n, r[h], Kx));
  };
  bf16x8 g[2][4], xa[4], xb[4];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int m = 0; m < 2; ++m) g[m][h] = ld(rg, bo(fo + 16 * m, r[h], Kg));
  ldx(xa, 0);
  l2 g8[2][2];
  int sg[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    sg[m] = mx_scale(mx_block(g[m], g8[m][0], g8[m][1]), lane);
    if (bias_tile) {
#pragma unroll
      for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) gs[m] += (float)g[m][h][e];
    }
  }
  // one X n-tile ahead: n-tile n + 1 loads while n converts (operand registers for two workgroups per CU)
#pragma unroll
  for (int n = 0; n < NX; ++n) {
    bf16x8 (&cur)[4] = (n & 1) ? xb : xa;
    bf16x8 (&nxt)[4] = (n & 1) ? xa : xb;
    if (n + 1 < NX) ldx(nxt, n + 1);
    l2 x0, x1;
    const int sx = mx_scale(mx_block(cur, x0, x1), lane);
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[m][n] = mx_mfma(g8[m][0], g8[m][1], x0, x1, acc[m][n], sg[m], sx);
  }
}

// One workgroup = tile td of layer L: 32 outputs × 32·NI inputs (NI = 2: two 32-wide input tiles
// sharing the G rows).  loss_block: this workgroup also finishes the loss (S, D, Z: its shape).
// MXW (NI = 2 only): the MX dW (mx_dw_chunk) in place of the bf16 MFMA loop; Bk % 128 == 0.
template <typename T, int MODE, int NI = 1, bool MXW = false>
__device__ __forceinline__ void wgrad_body(const LayerDev& L, const TileDesc td, int Bk, AdamArgs aa,
                                           const LossArgs& la, bool loss_block, int S, int D, int Z,
                                           float* red, float* dbp, SplitK sk = SplitK{1, 0, nullptr, nullptr, 0},
                                           const PeerArgs* px = nullptr) {
  static_assert(!MXW || (NI == 2 && std::is_same<T, __bf16>::value), "the MX dW: bf16 arena, 32 × 64 tiles");
  using V = typename Op<T>::V;
  constexpr int EPL = Op<T>::EPL, KC = Op<T>::KC;
  constexpr int NX = 2 * NI, TW = 32 * NI, LD = TW + 4;  // X fragments per chunk, tile width, image stride
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int r16 = lane & 15, kq = (lane >> 4) * EPL;
  const T* G = (const T*)L.gT;
  const T* X = (const T*)L.xT;
  const bool bias_tile = td.i0 == 0;
  // epilogue ownership: EPT = 2·NI weights per thread, all 512 threads (Adam's correctly rounded
  // sqrt and two divisions per weight are the epilogue's cost)
  constexpr int EPT = 2 * NI, TPR = TW / EPT;
  using VE = typename VecF<EPT>::T;
  const int o = tid / TPR, iv = (tid % TPR) * EPT;

  if (!CVAE_DIAG_WSTAMP_ENTRY) WSTAMP(0);
  const adam_f32x2 t_step = MODE == PM_ADAM ? adam_step_load(aa) : adam_f32x2{0.f, 0.f};
  f32x4 acc[2][NX];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < NX; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gs[2] = {0.f, 0.f};  // bias partials: Σ of this lane's G fragment elements
  // tile-major arena (aoff): this lane's 16-B pieces of rows o / i at batch offset kq of a chunk;
  // one chunk of KC batch rows advances KC/16 row tiles = (KC/16)·Kf·16 elements
  const int Kg = L.Np, Kx = L.Kp;
  const T* gp[2];
  const T* xp[NX];
#pragma unroll
  for (int m = 0; m < 2; ++m) gp[m] = G + aoff(td.o0 + m * 16 + r16, kq, Kg);
#pragma unroll
  for (int n = 0; n < NX; ++n) xp[n] = X + aoff(td.i0 + n * 16 + r16, kq, Kx);
  // this split's chunk range [c0, c0 + nk) (split-K; the whole batch when S == 1); this wave's
  // chunks: c0 + wave + WG_NW*j; PF chunks of loads kept in flight
  constexpr int KCH = MXW ? 128 : KC;  // batch rows per chunk
  const int nk_all = Bk / KCH, per = (nk_all + sk.S - 1) / sk.S;
  const int c0 = sk.s * per, nk = max(0, min(per, nk_all - c0));
  const int nmine = nk > wave ? (nk - wave + WG_NW - 1) / WG_NW : 0;
  // chunks in flight per wave: 4; 2 for 32 × 64 tiles, whose 6 operand vectors per chunk would
  // otherwise take the kernel past 128 VGPRs (one workgroup per CU instead of two)
  constexpr int PF = NI == 2 ? 2 : 4;
  V ga[PF][2], xb[PF][NX];
  auto load = [&](int u, int j) {  // unconditional, clamped to this wave's last chunk
    const size_t ct = (size_t)(c0 + wave + WG_NW * min(j, nmine > 0 ? nmine - 1 : 0)) * (KC / 16) * 16;
#pragma unroll
    for (int m = 0; m < 2; ++m) ga[u][m] = gld<V>(gp[m] + ct * Kg);
#pragma unroll
    for (int n = 0; n < NX; ++n) xb[u][n] = gld<V>(xp[n] + ct * Kx);
  };
  // the master state the epilogue updates (independent of the gradient), issued FIRST: the
  // compiler's waits inside loadn's paths then cover nothing but these loads, never the operands
  // MXW: after the MX loop instead (its operands need the registers; the loads then overlap the
  // cross-wave reduction)
  PreN<EPT> st = {};
  PreB sb = {0.f, 0.f, 0.f, -1};
  if (!MXW) {
    if (tid < 32 * TPR) st = loadn<MODE, EPT>(L, td.o0 + o, td.i0 + iv, aa);
    if (bias_tile && tid < 32) sb = loadb<MODE>(L, td.o0 + tid, aa);
  }
  if constexpr (MXW) {
    if (MODE == PM_ADAM) adam_resolve(aa, t_step);
    if (loss_block && wave == WG_NW - 1 && la.partials) finish_loss(la, S, D, Z);
    for (int jj = 0; jj < nmine; ++jj)
      mx_dw_chunk<NX>((const __bf16*)G, (const __bf16*)X, td.o0 + r16, td.i0 + r16, (c0 + wave + WG_NW * jj) * KCH,
                      Kg, Kx, acc, gs, bias_tile);
    if (tid < 32 * TPR) st = loadn<MODE, EPT>(L, td.o0 + o, td.i0 + iv, aa);
    if (bias_tile && tid < 32) sb = loadb<MODE>(L, td.o0 + tid, aa);
  } else {
#pragma unroll
  for (int u = 0; u < PF; ++u) load(u, u);
  // device-counter path: this step's Adam scalars (double pow), computed while the operands load
  if (MODE == PM_ADAM) adam_resolve(aa, t_step);
  if (loss_block && wave == WG_NW - 1 && la.partials) finish_loss(la, S, D, Z);
  for (int j0 = 0; j0 < nmine; j0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int j = j0 + u;
      if (j < nmine) {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < NX; ++n) acc[m][n] = mfma_chunk(ga[u][m], xb[u][n], acc[m][n]);
        if (bias_tile) {
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int e = 0; e < EPL; ++e) gs[m] += (float)ga[u][m][e];
        }
        if (j == 0) WSTAMP(7);
      }
      if (j + PF < nmine) load(u, j + PF);
    }
  }
  }  // bf16 loop
  WSTAMP(1);
  float* rw = red + wave * 32 * LD;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < NX; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) rw[(m * 16 + (lane >> 4) * 4 + i) * LD + n * 16 + r16] = acc[m][n][i];
  if (bias_tile) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      gs[m] += __shfl_xor(gs[m], 16, 64);
      gs[m] += __shfl_xor(gs[m], 32, 64);
      if (lane < 16) dbp[wave * 32 + m * 16 + lane] = gs[m];
    }
  }
  __syncthreads();
  WSTAMP(2);
  VE g4 = {};
  if (tid < 32 * TPR) {
#pragma unroll
    for (int w = 0; w < WG_NW; ++w) g4 += *(const VE*)(red + w * 32 * LD + o * LD + iv);
  }
  float db = 0.f;
  if (bias_tile && tid < 32) {
#pragma unroll
    for (int w = 0; w < WG_NW; ++w) db += dbp[w * 32 + tid];
  }
  if (px) {  // peer exchange (cvae_peer.h): PM_GRAD = a non-owner's tile, PM_ADAM = the owner's
    if (MODE == PM_GRAD) {
      px_push(*px, sk.tile, o, iv, g4, db, bias_tile);
      return;
    }
    __syncthreads();  // every wave has read red (g4): dbp[0] becomes the wait flag
    if (!px_gather(*px, aa.ctr, sk.tile, o, iv, g4, db, bias_tile, (int*)dbp)) return;
    if (!px->ragged) {
      g4 = g4 * aa.grad_scale;
      db = db * aa.grad_scale;
    }
  }
  if (sk.S > 1) {  // split-K: publish this split's partial; the last of the S blocks finishes the tile
    const int PW = sk.pw ? sk.pw : 32 * TW + 32;
    static_assert(EPT == 2 || EPT == 4, "partial vectors of 8 or 16 B");
    float* mine = sk.ws + ((size_t)sk.tile * sk.S + sk.s) * PW;
    if (tid < 32 * TPR) {
      if constexpr (EPT == 2)
        __hip_atomic_store((uint64_t*)(mine + o * TW + iv), __builtin_bit_cast(uint64_t, g4), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      else
        for (int c = 0; c < EPT; c += 2)
          __hip_atomic_store((uint64_t*)(mine + o * TW + iv + c),
                             __builtin_bit_cast(uint64_t, VecF<2>::T{g4[c], g4[c + 1]}), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    }
    if (bias_tile && tid < 32)
      __hip_atomic_store((unsigned*)(mine + 32 * TW + tid), __builtin_bit_cast(unsigned, db), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    // the hand-off in MI355X_MICROARCH.md's sc1 form (its table of valid hand-offs, first row):
    // every partial store above is sc1 (relaxed agent-scope atomic stores), every storing wave
    // drains them (the asm wait is also a compiler barrier: no store sinks past it), the block joins
    // a barrier, ONE lane adds to the tile's ticket, and the block whose add returned S-1 reads the
    // partials with sc1 loads only (relaxed agent-scope atomic loads below).  Agent-scope
    // release/acquire fences here — an L2 write-back and an L1 invalidate per block, ~1.7 µs each —
    // took the split-K dW from 44 to 486 µs at B = 16384 (profiles/r03i/bsweep_fences.md).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(sk.tickets + sk.tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      dbp[0] = __builtin_bit_cast(float, old);
    }
    __syncthreads();
    if (__builtin_bit_cast(unsigned, dbp[0]) != (unsigned)(sk.S - 1)) return;  // block-uniform
    // the last arriver: Σ of the S partials in split order
    g4 = VE{};
    db = 0.f;
    for (int k = 0; k < sk.S; ++k) {
      const float* pk = sk.ws + ((size_t)sk.tile * sk.S + k) * PW;
      if (tid < 32 * TPR) {
#pragma unroll
        for (int c = 0; c < EPT; c += 2) {
          const uint64_t u = __hip_atomic_load((const uint64_t*)(pk + o * TW + iv + c), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
          const typename VecF<2>::T v2 = __builtin_bit_cast(typename VecF<2>::T, u);
          g4[c] += v2[0];
          g4[c + 1] += v2[1];
        }
      }
      if (bias_tile && tid < 32)
        db += __builtin_bit_cast(float, __hip_atomic_load((const unsigned*)(pk + 32 * TW + tid), __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT));
    }
    if (tid == 0) sk.tickets[sk.tile] = 0u;  // every split has added: reset for the next launch
  }
  __syncthreads();  // red becomes the image of the new weights
  const float nb = tile_epilogue<T, MODE, WG_THREADS, EPT, NI>(L, td.o0, td.i0, st, sb, g4, db, aa, red);
  if (MODE == PM_ADAM && px) px_broadcast<T, WG_THREADS>(*px, L, td.o0, td.i0, red, nb);
#if CVAE_DIAG_STAMPS
  __syncthreads();
  WSTAMP(3);
#endif
}

// generic configurations: tile descriptors and layer records from memory
// grid = ntiles × sk.S (split-major: split s owns blocks [s·ntiles, (s+1)·ntiles))
// NI2: the tile list holds 32 × 64 tiles (TileDesc::ni == 2) beside 32 × 32 ones — a large tile
// list (BASELINE cfg5: 868 tiles of 32 × 32 for 512 workgroup slots) then needs fewer workgroups
// and re-reads fewer arena rows (a tile reads 32 G rows + 32·ni X rows of the whole batch)
// (launch bounds: 4 waves per SIMD = two workgroups per CU)
template <typename T, int MODE, bool NI2 = false>
__global__ __launch_bounds__(WG_THREADS, 4) void wgrad_kernel(NetDev net, const TileDesc* __restrict__ tiles,
                                                           int Bk, AdamArgs aa, LossArgs la, SplitK sk) {
  __shared__ __attribute__((aligned(16))) WgradLds<NI2 ? 2 : 1> sh;
  if (CVAE_DIAG_WSTAMP_ENTRY) WSTAMP(0);
  const int ntiles = gridDim.x / sk.S;
  sk.s = blockIdx.x / ntiles;
  sk.tile = blockIdx.x - sk.s * ntiles;
  const TileDesc td = tiles[sk.tile];
  if constexpr (NI2) {
    if (td.ni == 2) {  // block-uniform
      wgrad_body<T, MODE, 2>(net.L[td.layer], td, Bk, aa, la, blockIdx.x == 0, net.S, net.D, net.Z, sh.red,
                                    sh.dbp, sk);
      return;
    }
  }
  wgrad_body<T, MODE>(net.L[td.layer], td, Bk, aa, la, blockIdx.x == 0, net.S, net.D, net.Z, sh.red, sh.dbp, sk);
}

// Adam from a (reduced) gradient buffer, or repack of the operand copies.
template <typename T, int MODE>
__device__ __forceinline__ void param_body(const LayerDev& L, const TileDesc& td, AdamArgs aa, float* wt) {
  const int tid = threadIdx.x;
  const adam_f32x2 t_step = MODE == PM_ADAM ? adam_step_load(aa) : adam_f32x2{0.f, 0.f};  // first: in-order vmcnt
  const PreN<4> st = loadn<MODE, 4>(L, td.o0 + (tid >> 3), td.i0 + (tid & 7) * 4, aa);
  PreB sb = {0.f, 0.f, 0.f, -1};
  if (td.i0 == 0 && tid < 32) sb = loadb<MODE>(L, td.o0 + tid, aa);
  f32x4 g4 = {0.f, 0.f, 0.f, 0.f};
  float db = 0.f;
  if (MODE == PM_ADAM) {
#pragma unroll
    for (int c = 0; c < 4; ++c) g4[c] = c < st.nv ? aa.grads[st.base + c * st.stride] * aa.grad_scale : 0.f;
    const int ob = td.o0 + tid;
    if (td.i0 == 0 && tid < 32 && ob < L.N && L.has_bias) {
      const int seg = (L.nseg == 2 && ob >= L.seg_rows0) ? 1 : 0;
      db = aa.grads[L.pb[seg] + (seg ? ob - L.seg_rows0 : ob)] * aa.grad_scale;
    }
    adam_resolve(aa, t_step);  // its first use: after every state load has been issued
  }
  tile_epilogue<T, MODE, CVAE_THREADS, 4>(L, td.o0, td.i0, st, sb, g4, db, aa, wt);
}

template <typename T, int MODE>
__global__ __launch_bounds__(CVAE_THREADS) void param_kernel(NetDev net, const TileDesc* __restrict__ tiles,
                                                             AdamArgs aa) {
  __shared__ __attribute__((aligned(16))) float wt[32 * WT_LD];
  const TileDesc td = tiles[blockIdx.x];
  param_body<T, MODE>(net.L[td.layer], td, aa, wt);
}

// CVAE_FP8: the per-layer weight scale of the e4m3 forward operand (cvae_device.h F8Scale), one
// block per layer: s = 2^floor(log2(448 / (4·max|W|))) — a power of two (exact to apply and to
// undo), with 4x headroom so Adam's drift between packs stays inside e4m3's range (beyond it the
// conversion saturates).  Run by cvae_pack_weights before the pack; Adam then writes Wf with s.
__global__ __launch_bounds__(CVAE_THREADS) void f8_scale_kernel(NetDev net, const float* __restrict__ params) {
  const LayerDev& L = net.L[blockIdx.x];
  if (!L.f8) return;
  float m = 0.f;
  const int n = L.N * L.K;
  for (int j = threadIdx.x; j < n; j += CVAE_THREADS) {
    const int o = j / L.K, i = j - o * L.K;
    const int seg = (L.nseg == 2 && o >= L.seg_rows0) ? 1 : 0;
    m = fmaxf(m, fabsf(params[L.wt ? L.pw[0] + (int64_t)i * L.N + o
                                   : L.pw[seg] + (int64_t)(seg ? o - L.seg_rows0 : o) * L.K + i]));
  }
  __shared__ float red[CVAE_THREADS];
  red[threadIdx.x] = m;
  __syncthreads();
  for (int k = CVAE_THREADS / 2; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + k]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float amax = red[0];
    const float sc = amax > 0.f ? exp2f(floorf(log2f(F8_MAX / (4.f * amax)))) : 1.f;
    F8Scale* hd = (F8Scale*)((char*)L.Wf - sizeof(F8Scale));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    gst<f32x2>(&hd->s, f32x2{sc, 1.f / sc});  // vector store
  }
}

