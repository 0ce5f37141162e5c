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
// Structure: a compact LAYER INTERPRETER.  The host builds a step table (one
// entry per GEMM: operand buffers, weights, epilogue kind and targets); the
// kernel runs ONE instance of the GEMM loop over it, epilogues chosen by a
// wave-uniform switch.  A fully inlined version of the same chain compiled to
// 90 KB of straight-line code that ran once per launch — larger than the
// instruction cache — and spent ~3 µs per layer fetching instructions; this
// version keeps the hot code small and re-executed.
//
// GEMM core: Y[R×Np] = X[R×Kp]·Wᵀ, X from LDS (A operand, ds_read_b128), W streamed
// from L2 straight into registers (B operand), double-buffered across K blocks,
// column groups and layers (see `dense`).  MFMA 16x16x32 bf16 or 4×16x16x4 f32.
// ReLU masks are kept as bits in LDS for the backward pass.  Barriers between
// steps are LDS-only (`lds_barrier`): global stores never drain at a barrier.
#pragma once
#include "cvae_device.h"

enum { RC_TRAIN = 0, RC_FWD = 1, RC_DECODE = 2 };

// Batch rows per workgroup.  The swapped GEMM's MFMA N dimension is 16 batch columns; with
// R < 16 (4 or 8) lanes r16 >= R recompute row r16 % R — identical values to identical
// addresses — which wastes MFMA columns but multiplies the workgroups of a launch by 16/R:
// the chain is latency-bound, so more concurrent row tiles is what raises throughput.
#ifndef CVAE_ROWS
#define CVAE_ROWS 16
#endif
template <typename T> struct RowsPerTile { static constexpr int R = CVAE_ROWS; };
static_assert(CVAE_ROWS == 4 || CVAE_ROWS == 8 || CVAE_ROWS % 16 == 0, "row tile: 4, 8 or a multiple of 16");

// Waves per row-chain workgroup.  8 = two waves per SIMD: each step's column groups are
// spread over twice the waves (16-feature groups, one n-tile each), and the SIMD overlaps one
// wave's load / LDS / barrier latency with the other's issue.  4 = one wave per SIMD with
// 32-feature groups (two n-tiles).
#ifndef CVAE_RC_WAVES
#define CVAE_RC_WAVES 8
#endif
constexpr int RC_NW = CVAE_RC_WAVES;
constexpr int RC_THREADS = 64 * RC_NW;
constexpr int RC_NT = RC_NW >= 8 ? 1 : 2;  // n-tiles (16 output features) per column group
constexpr int RC_GW = 16 * RC_NT;          // column-group width
static_assert(RC_NW == 4 || RC_NW == 8, "row chain: 4 or 8 waves");

// exact a / b for 0 <= a < 2^22 and small b, from a precomputed 1/b: (a + ½)/b is at least ½/b
// away from an integer, far more than the float rounding error — no integer-division sequence
__device__ __forceinline__ int fdiv(int a, float inv_b) { return (int)(((float)a + 0.5f) * inv_b); }

// LDS row of MFMA tile m, lane row r16
template <int R>
__device__ __forceinline__ int tile_row(int m, int r16) { return R >= 16 ? m * 16 + r16 : (r16 & (R - 1)); }

// Diagnostic builds only (scripts/diag_*.sh): drop the arena stores to price them /
// record per-step time stamps.  Results are wrong under NOSTORE; the shipped library
// defines neither.
#ifndef CVAE_DIAG_NOSTORE
#define CVAE_DIAG_NOSTORE 0
#endif
#ifndef CVAE_DIAG_STAMPS
#define CVAE_DIAG_STAMPS 0
#endif
#ifndef CVAE_DIAG_SUB
#define CVAE_DIAG_SUB 0
#endif
// ablations (timing only, results wrong): no weight loads / no epilogue / no MFMAs
#ifndef CVAE_DIAG_NOWLOAD
#define CVAE_DIAG_NOWLOAD 0
#endif
#ifndef CVAE_DIAG_NOEPI
#define CVAE_DIAG_NOEPI 0
#endif
#ifndef CVAE_DIAG_NOMFMA
#define CVAE_DIAG_NOMFMA 0
#endif
#ifndef CVAE_DIAG_NOLDSW
#define CVAE_DIAG_NOLDSW 0
#endif
#ifndef CVAE_DIAG_NOBAR
#define CVAE_DIAG_NOBAR 0
#endif
#ifndef CVAE_DIAG_NOBIAS
#define CVAE_DIAG_NOBIAS 0
#endif
#if CVAE_DIAG_SUB
// [block][wave][step][5]: entry, weights arrived, MFMAs done, epilogue done, barrier passed
__device__ unsigned long long* g_sub;
__device__ int g_sub_step;
#define SUBSTAMP(k)                                                                                     \
  do {                                                                                                  \
    if ((threadIdx.x & 63) == 0 && g_sub && g_sub_step < 32)                                            \
      g_sub[((blockIdx.x * RC_NW + (threadIdx.x >> 6)) * 32 + g_sub_step) * 5 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define SUBSTAMP(k) do { } while (0)
#endif

// LDS buffers a step can read or write
enum { B_NONE = -1, B_XIN = 0, B_P0 = 1, B_P1 = 2, B_HC = 3, B_DEC = 4, B_CIN = 5, B_CLS = 6 };
// epilogue kinds; post-step element-wise phases
enum { E_RELU = 0, E_FC = 1, E_LOSS = 2, E_RECON = 3, E_BWD = 4, E_D0B = 5, E_FCB = 6 };

// One step of the interpreter as the host builds it (cvae_capi.hip build_steps) ...
struct StepSpec {
  const void* W;     // weight operand ~[Np][Kp] in fragment order (forward Wf or backward Wb)
  int bias_off;      // offset of this step's bias in the LDS bias copy (-1: zeros, backward)
  void* g1;          // arena destination (feature-major), nullable
  void* g2;
  int Kp, Np;        // reduction / output dims (padded)
  int N;             // real output columns
  int xbuf;          // LDS source
  int epi;           // E_*
  int mask_out;      // forward: ReLU mask index to set (-1 none)
  int mask_in;       // backward: ReLU mask index to apply
  int dst1, off1;    // LDS destinations (B_NONE = none) and column offsets
  int dst2, off2;
  int goff1, goff2;  // arena row offsets of g1 / g2
  int concat;        // skip columns >= N (destination is part of a concatenation)
  int linear;        // forward step without ReLU and mask (the class embedding)
  int hc_out;        // inference: also write h_c (fp32) to RowArgs::hc_out
  int kf1, kf2;      // feature rows of the g1 / g2 arena matrices (aoff)
  int f8;            // CVAE_FP8 forward step (e4m3 W and X)
};

// ... and as the kernel reads it: 64 B, copied into LDS by the prologue and read back every step
// with wave-uniform LDS reads + readfirstlane.  (Scalar loads share lgkmcnt with LDS and return
// out of order: a descriptor fetched with s_load makes the step's first LDS wait also wait for
// an L2 round trip, on every step of every launch.)
struct StepDesc {
  const void* W;
  void* g1;
  void* g2;
  int Kp, Np, N, bias_off;
  int code;          // xbuf | epi<<4 | (dst1+1)<<8 | (dst2+1)<<12 | concat<<16 | hc_out<<17 | linear<<18 | (mask_out+1)<<20 | (mask_in+1)<<26
  int off1, off2;
  int goff;          // goff1 | goff2 << 16
  int kf1, kf2;      // feature rows of the g1 / g2 arena matrices
};
static_assert(sizeof(StepDesc) == 64, "StepDesc is 4 x 16 B");

inline StepDesc encode_step(const StepSpec& s) {
  StepDesc d{};
  d.W = s.W; d.g1 = s.g1; d.g2 = s.g2;
  d.Kp = s.f8 ? (s.Kp / 2) | (1 << 30) : s.Kp;  // f8: the weight stream counts 64-wide K pairs
  d.Np = s.Np; d.N = s.N; d.bias_off = s.bias_off;
  d.code = s.xbuf | (s.epi << 4) | ((s.dst1 + 1) << 8) | ((s.dst2 + 1) << 12) | (s.concat << 16) |
           (s.hc_out << 17) | (s.linear << 18) | ((s.mask_out + 1) << 20) | ((s.mask_in + 1) << 26);
  d.off1 = s.off1; d.off2 = s.off2;
  d.goff = s.goff1 | (s.goff2 << 16);
  d.kf1 = s.kf1; d.kf2 = s.kf2;
  return d;
}

struct RowArgs {
  const void* x;          // (N_total, S, D) operand dtype (fp32 with x_f32)
  const int64_t* idx;     // optional row gather
  int batch;
  int nsteps;
  const StepDesc* steps;  // step table of this mode (device)
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
  unsigned long long* stamps;  // diagnostic builds only
  int x_relative;         // 1: x is relative, condition = start_in (no transform)
  int x_f32;              // 1: x is fp32 whatever T (relative transform in fp32, one rounding)
  int64_t eps_row0;       // Philox rows are keyed by the GLOBAL row eps_row0 + b (data parallelism)
  uint64_t* ctr;          // device step counters (cvae.h): offset = ctr[0]; block 0 begins step ctr[1] + 1
  int adam_pre;           // ... and precomputes that step's Adam scalars into ctr[2] (lr, betas below)
  double lr, beta1, beta2;
  float* eps_out;         // FWD: the eps each row used (fp32 (batch, Z), nullable)
  // external-gradient backward (cvae_backward): the loss gradient is given, not computed
  int ext;
  const float* d_recon;   // (batch, S, D) fp32, nullable = 0
  const float* d_mu;      // (batch, Z)
  const float* d_lv;      // (batch, Z)
  const float* d_hc;      // (batch, H)
  const int* classes;     // cfg4: class id per row of x (gathered by idx like x); NULL = class 0
  int ncls, cdim;         // cfg4: n_classes, class_dim (0 for the reference model)
};

// Philox offset of this launch's eps draws: the device counter when given (a replayable step)
__device__ __forceinline__ uint64_t rng_offset(const RowArgs& a) { return a.ctr ? gld<uint64_t>(a.ctr) : a.offset; }

struct LdsPlan {
  int sx, sp, shc, sdec, scin;   // row strides (elements of T)
  int mw;                        // mask words per row
  int oXin, oP0, oP1, oHc, oDec, oCin, oMuLv, oDz, oU, oRch0, oGd0, oStart, oRow, oMask, oPart, oBias, oSteps;
  int oF8;                       // CVAE_FP8: e4m3 image of a wide step's input (R x F8_LD bytes)
  int scls, oCls, oDce;          // cfg4: one-hot class input (R x scls T), decoder share of de (R x cls_dim fp32)
  int total;
};
// CVAE_FP8 steps with K <= 256 convert their input once per step into an e4m3 LDS image in
// fragment order ([row][chunk][q][8 B]; row stride 288 B keeps 8 rows x 4 lane groups on
// distinct banks) instead of in every wave and column group (measured at cfg5: row chain 140 ->
// 131 us).  Wider inputs (encoder L1, decoder L0) convert per chunk (measured: an image in the
// dead ping-pong buffer bought nothing).
constexpr int F8_IMG_K = 256, F8_LD = F8_IMG_K + 32;

__host__ __device__ inline int rup(int v, int a) { return (v + a - 1) / a * a; }

__host__ __device__ inline int n_masks(const NetDev& n) { return 2 + n.n_enc + (n.n_dec - 1); }

__host__ __device__ inline LdsPlan lds_plan(const NetDev& n, int R, int tsize) {
  LdsPlan p;
  const int pad = 16 / tsize;  // +16 B per row: 16-B LDS reads of 16 consecutive rows hit distinct banks
  p.sx = n.Ip + pad;
  p.sp = (n.Hp > n.Zp2 ? n.Hp : n.Zp2) + pad;
  p.shc = n.Hcp + pad;
  p.sdec = n.ZHp + pad;
  p.scin = n.Cp + pad;
  p.mw = n.Hp / 4;  // mask bytes per row (4 features per byte)
  int o = 0;
  auto take = [&](int bytes) { int r = o; o += rup(bytes, 16); return r; };
  p.oXin = take(R * p.sx * tsize);
  p.oP0 = take(R * p.sp * tsize);
  p.oP1 = take(R * p.sp * tsize);
  p.oHc = take(R * p.shc * tsize);
  p.oDec = take(R * p.sdec * tsize);
  p.oCin = take(R * p.scin * tsize);
  p.oMuLv = take(R * n.Zp2 * 4);
  p.oDz = take(R * n.Z * 4);
  const int ub = (2 * n.S > n.H ? 2 * n.S : n.H) * R * 4;
  p.oU = take(ub);
  p.oRch0 = p.oU;
  p.oGd0 = p.oU + R * n.S * 4;
  p.oStart = take(R * 2 * 4);
  p.oRow = take(R * 8);
  p.oMask = take(n_masks(n) * R * p.mw);
  p.oPart = take(RC_NW * 8 * 4);
  p.oBias = take((n.nbias + 4) * 4);  // + 4 zero floats: the bias of backward steps
  p.oSteps = take(64 * (int)sizeof(StepDesc));
  p.oF8 = take(n.dtype == 2 /* CVAE_FP8 */ ? R * F8_LD : 0);
  p.scls = n.Clsp + pad;
  p.oCls = take(n.n_cls ? R * p.scls * tsize : 0);
  p.oDce = take(n.n_cls ? R * n.cls_dim * 4 : 0);
  p.total = o;
  return p;
}

// ---------------------------------------------------------------- weight-stream GEMM
// A wave owns 32-column groups g = wave, wave+4, ...; each group's K range is cut into
// blocks of NKB chunks held in a register block.  The weight stream is double-buffered
// across blocks, groups AND steps: while block i is multiplied, block i+1 — possibly of the
// next group, or the first block of the NEXT step — is already in flight in `pre`.
// Every load is unconditional (the source is selected, chunk indices clamped): a load under
// a branch makes hipcc wait vmcnt(0) (cdna_hip_programming.md §5 trap (c)).  Loads are
// issued before the epilogue's global stores, so waiting for them never waits for those
// stores (vmcnt retires in order).
constexpr int NKB = 4;
#ifndef CVAE_LATE_PREFETCH
#define CVAE_LATE_PREFETCH 0
#endif

template <typename T>
struct WBlock {
  typename Op<T>::V b[NKB][RC_NT];
};

template <typename T>
__device__ __forceinline__ void load_block(WBlock<T>& wb, const T* __restrict__ W, int Kp, int Np, int g, int blk) {
  using V = typename Op<T>::V;
  constexpr int EPL = Op<T>::EPL, KC = Op<T>::KC;
  const int lane = threadIdx.x & 63;
  const int nk = Kp / KC, ng = Np / RC_GW;
  g = min(g, ng - 1);
  // fragment order (frag_off): n-tile t, chunk kc → 1 KB at ((t * nk + kc) * 64 + lane) * EPL
  const T* w0 = W + (size_t)lane * EPL;
#pragma unroll
  for (int u = 0; u < NKB; ++u) {
    const int kc = min(blk * NKB + u, nk - 1);
#pragma unroll
    for (int j = 0; j < RC_NT; ++j) {
      const int t = g * RC_NT + j;
      wb.b[u][j] = CVAE_DIAG_NOWLOAD ? V{} : gld<V>(w0 + (size_t)(t * nk + kc) * 64 * EPL);
    }
  }
}

// B-operand fragment of one row-major activation row for K chunk starting at p: lane group q takes
// the chunk positions frag_k(q, e) (two 8-B halves for bf16, matching the weight fragments)
template <typename T>
__device__ __forceinline__ typename Op<T>::V xchunk(const T* p, int q);
template <>
__device__ __forceinline__ f32x4 xchunk<float>(const float* p, int q) { return *(const f32x4*)(p + 4 * q); }
template <>
__device__ __forceinline__ bf16x8 xchunk<__bf16>(const __bf16* p, int q) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const bf16x4 lo = *(const bf16x4*)(p + 4 * q), hi = *(const bf16x4*)(p + 16 + 4 * q);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// epi(row, f0, v) receives v[i] = Y[row][f0 + i], i = 0..3: the MFMA computes Yᵀ = W·Xᵀ
// (A = weights, B = activations), so a lane's accumulator holds FOUR CONSECUTIVE FEATURES of
// one row — one 8/16-B LDS store, one float4 bias and one 4-bit mask nibble per call.
// BIAS: the group's 4 bias values are read from LDS at the top of the item — before the X reads
// and MFMAs — so their latency hides there instead of opening the epilogue.
template <typename T, int R, bool BIAS, class Epi>
__device__ __forceinline__ void dense(const T* __restrict__ Xs, int ldx, const T* __restrict__ W, int Kp, int Np,
                                      WBlock<T>& pre, const T* nW, int nKp, int nNp, const float* biasL,
                                      Epi&& epi, bool f8 = false, float inv_s = 1.f,
                                      const uint8_t* f8img = nullptr) {
  using V = typename Op<T>::V;
  constexpr int EPL = Op<T>::EPL, KC = Op<T>::KC, MT = R >= 16 ? R / 16 : 1;
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int r16 = lane & 15;
  const int NG = Np / RC_GW, nk = Kp / KC, nblk = (nk + NKB - 1) / NKB;
  const int ng_mine = NG > wave ? (NG - wave + RC_NW - 1) / RC_NW : 0;
  const int nitems = ng_mine * nblk;
  if (nitems == 0) {  // idle in this step: still stream the next step's first block
    if (nW) load_block(pre, nW, nKp, nNp, wave, 0);
    return;
  }
  f32x4 acc[RC_NT][MT];
#pragma unroll
  for (int j = 0; j < RC_NT; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (group, block) of the current and the next item, advanced without integer division
  int gi = 0, blk = 0;
  for (int it = 0; it < nitems; ++it) {
    const bool wrap = blk + 1 == nblk;
    const int gi_n = wrap ? gi + 1 : gi, blk_n = wrap ? 0 : blk + 1;
    const int g = wave + gi * RC_NW;
    f32x4 b4[RC_NT];
#pragma unroll
    for (int j = 0; j < RC_NT; ++j)
      b4[j] = BIAS ? *(const f32x4*)(biasL + g * RC_GW + j * 16 + (lane >> 4) * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    const WBlock<T> cur = pre;
#if CVAE_DIAG_SUB
    if (it == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      SUBSTAMP(1);
    }
#endif
    // next item: this step's next block/group, else the next step's first block
    auto prefetch = [&]() {
      const bool same = it + 1 < nitems;
      const T* W2 = same ? W : (nW ? nW : W);
      const int Kp2 = same ? Kp : (nW ? nKp : Kp);
      const int Np2 = same ? Np : (nW ? nNp : Np);
      const int g2 = same ? wave + gi_n * RC_NW : wave;
      const int blk2 = same ? blk_n : 0;
      load_block(pre, W2, Kp2, Np2, g2, blk2);
    };
    if (!CVAE_LATE_PREFETCH) prefetch();
    // all LDS reads of the block first (one lgkmcnt wait per block, not per chunk), then the
    // MFMAs unconditionally: chunks past K read a clamped (valid) address and are zeroed, so a
    // short block costs a few idle MFMAs instead of branches and per-chunk waits
    bool f8_done = false;
    if constexpr (EPL == 8) {
      if (f8) {  // CVAE_FP8 forward step: a 16-B fragment = two 32-wide K chunks of e4m3 (Kp, nk count K/64 pairs)
        // chunk pairs past K are skipped (uniform branches; no loads inside): a 128-wide K is
        // 2 pairs of a 4-pair block, and issuing the idle half cost 25 % more MFMAs per launch
        long x8[NKB][MT][2];
#pragma unroll
        for (int u = 0; u < NKB; ++u) {
          const int kc = min(blk * NKB + u, nk - 1);
          if (blk * NKB + u >= nk) continue;
#pragma unroll
          for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh)
              x8[u][m][hh] = f8img ? *(const long*)(f8img + tile_row<R>(m, r16) * F8_LD + (kc * 2 + hh) * KC + (lane >> 4) * 8)
                                   : f8x8(xchunk<T>(Xs + tile_row<R>(m, r16) * ldx + kc * 2 * KC + hh * KC, lane >> 4));
        }
#pragma unroll
        for (int u = 0; u < NKB; ++u) {
          if (blk * NKB + u >= nk) continue;
#pragma unroll
          for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int j = 0; j < RC_NT; ++j) {
              typedef long l2 __attribute__((ext_vector_type(2)));
              const l2 wa = __builtin_bit_cast(l2, cur.b[u][j]);
              if (!CVAE_DIAG_NOMFMA) {
                acc[j][m] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(wa[0], x8[u][m][0], acc[j][m], 0, 0, 0);
                acc[j][m] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(wa[1], x8[u][m][1], acc[j][m], 0, 0, 0);
              }
            }
        }
        f8_done = true;
      }
    }
    if (!f8_done) {
      V xa[NKB][MT];
#pragma unroll
      for (int u = 0; u < NKB; ++u) {
        const int kc = min(blk * NKB + u, nk - 1);
#pragma unroll
        for (int m = 0; m < MT; ++m) xa[u][m] = xchunk<T>(Xs + tile_row<R>(m, r16) * ldx + kc * KC, lane >> 4);
      }
#pragma unroll
      for (int u = 0; u < NKB; ++u) {
        const bool on = blk * NKB + u < nk;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const V xb = on ? xa[u][m] : V{};
#pragma unroll
          for (int j = 0; j < RC_NT; ++j)
            if (!CVAE_DIAG_NOMFMA) acc[j][m] = mfma_chunk(cur.b[u][j], xb, acc[j][m]);
        }
      }
    }
    // issued behind the MFMAs: all waves issue their loads right after a barrier, and the CU's
    // vector-memory path (~64 B/clk) takes hundreds of cycles to accept them; placed here the
    // wave's MFMAs already run while its load instructions queue
    if (CVAE_LATE_PREFETCH) prefetch();
#if CVAE_DIAG_SUB
    if (it == 0) SUBSTAMP(2);
#endif
    if (blk == nblk - 1) {
#pragma unroll
      for (int j = 0; j < RC_NT; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          epi(tile_row<R>(m, r16), g * RC_GW + j * 16 + (lane >> 4) * 4, f8 ? acc[j][m] * inv_s : acc[j][m], b4[j]);
          acc[j][m] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
#if CVAE_DIAG_SUB
      if (it == nblk - 1) SUBSTAMP(3);
#endif
    }
    gi = gi_n;
    blk = blk_n;
  }
}

// Workgroup barrier for LDS hand-offs only: no vmcnt drain, so global stores and the weight
// prefetch stay in flight across it (nothing in this kernel reads back its global stores).
__device__ __forceinline__ void lds_barrier() {
  if (CVAE_DIAG_NOBAR) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <typename T>
__device__ __forceinline__ void st4(T* p, f32x4 v) {
  if (!CVAE_DIAG_NOSTORE) store4(p, v);
}

// 4 consecutive T values from floats: one 8-B (bf16) / 16-B (fp32) LDS or global store
__device__ __forceinline__ void put4(float* p, f32x4 v) { *(f32x4*)p = v; }
__device__ __forceinline__ void put4(__bf16* p, f32x4 v) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 h;
  h[0] = (__bf16)v[0]; h[1] = (__bf16)v[1]; h[2] = (__bf16)v[2]; h[3] = (__bf16)v[3];
  *(bf16x4*)p = h;
}
__device__ __forceinline__ f32x4 get4(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ f32x4 get4(const __bf16* p) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const bf16x4 h = *(const bf16x4*)p;
  return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
}
__device__ __forceinline__ void gstore4(float* p, f32x4 v) { gst<f32x4>(p, v); }
__device__ __forceinline__ void gstore4(__bf16* p, f32x4 v) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 h;
  h[0] = (__bf16)v[0]; h[1] = (__bf16)v[1]; h[2] = (__bf16)v[2]; h[3] = (__bf16)v[3];
  gst<bf16x4>(p, h);
}
// feature-major arena store of 4 consecutive features of one row (4 element stores)
template <typename T>
__device__ __forceinline__ void put4T(T* base, int Bp, f32x4 v) {
  if (CVAE_DIAG_NOSTORE) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) gst<T>(base + (size_t)i * Bp, to_t<T>(v[i]));
}
// Feature-major arena store of one lane's 4 consecutive features as ONE wide store.  The 4
// lanes q = lane & 3 of a quad hold rows r0..r0+3 (r0 = row & ~3) of the same 4 features; a 4x4
// transpose across the quad (two DPP quad_perm exchanges) leaves lane q with feature f0+q of
// rows r0..r0+3, contiguous in the arena: one 8-B (bf16) / 16-B (fp32) store instead of four
// 2/4-B ones.  Per-CU store issue is ~one wave store instruction per 25 cycles whatever its width
// (MI355X_MICROARCH.md, plain-store rate), so the instruction count is what costs.
__device__ __forceinline__ uint32_t dpp_xor1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
}
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 h;
  h[0] = (__bf16)a;
  h[1] = (__bf16)b;
  return __builtin_bit_cast(uint32_t, h);
}
// arena matrix mat (Kf feature rows), features f0..f0+3; brow = this lane's batch row
// (brow & 3 == lane & 3)
__device__ __forceinline__ void put4Tq(__bf16* mat, int Kf, int f0, int brow, f32x4 y) {
  if (CVAE_DIAG_NOSTORE) return;
  const int lane = threadIdx.x & 63;
  const bool b1 = lane & 1, b2 = lane & 2;
  const uint32_t P0 = pack_bf16(y[0], y[1]), P1 = pack_bf16(y[2], y[3]);
  // distance 2: rows {0,1} keep features {0,1} and take rows {2,3}'s; rows {2,3} the converse
  const uint32_t R = dpp_xor2(b2 ? P0 : P1);
  const uint32_t D0 = b2 ? R : P0, D1 = b2 ? P1 : R;
  // distance 1, 16-bit halves: even lanes send (hi D0, hi D1), odd lanes (lo D0, lo D1)
  const uint32_t R2 = dpp_xor1(b1 ? __builtin_amdgcn_perm(D1, D0, 0x05040100u)
                                  : __builtin_amdgcn_perm(D1, D0, 0x07060302u));
  const uint32_t Q0 = b1 ? __builtin_amdgcn_perm(D0, R2, 0x07060100u) : __builtin_amdgcn_perm(R2, D0, 0x05040100u);
  const uint32_t Q1 = b1 ? __builtin_amdgcn_perm(D1, R2, 0x07060302u) : __builtin_amdgcn_perm(R2, D1, 0x07060100u);
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  gst<u32x2>(mat + aoff(f0 + (lane & 3), brow & ~3, Kf), u32x2{Q0, Q1});
}
__device__ __forceinline__ void put4Tq(float* mat, int Kf, int f0, int brow, f32x4 y) {
  if (CVAE_DIAG_NOSTORE) return;
  const int lane = threadIdx.x & 63;
  const bool b1 = lane & 1, b2 = lane & 2;
  auto u = [](float f) { return __builtin_bit_cast(uint32_t, f); };
  auto f = [](uint32_t v) { return __builtin_bit_cast(float, v); };
  // distance 2: rows {0,1} send features {2,3}, rows {2,3} send features {0,1}
  const uint32_t Ra = dpp_xor2(u(b2 ? y[0] : y[2])), Rb = dpp_xor2(u(b2 ? y[1] : y[3]));
  const float A0 = b2 ? f(Ra) : y[0], A1 = b2 ? f(Rb) : y[1];
  const float A2 = b2 ? y[2] : f(Ra), A3 = b2 ? y[3] : f(Rb);
  // distance 1: even lanes send (A1, A3), odd lanes (A0, A2)
  const uint32_t Rc = dpp_xor1(u(b1 ? A0 : A1)), Rd = dpp_xor1(u(b1 ? A2 : A3));
  const f32x4 q = b1 ? f32x4{f(Rc), A1, f(Rd), A3} : f32x4{A0, f(Rc), A2, f(Rd)};
  gst<f32x4>(mat + aoff(f0 + (lane & 3), brow & ~3, Kf), q);
}

// the 4 ReLU bits of features f0..f0+3 (f0 % 4 == 0) of one row: one byte per 4-feature group
__device__ __forceinline__ uint32_t mask4(const uint8_t* mk, int mw, int row, int f0) {
  return mk[row * mw + (f0 >> 2)];
}

// F8: the CVAE_FP8 instantiation (bf16 activations, e4m3 forward steps); without it every step's
// fp8 flag is a constant false and the fp8 code folds away.
template <typename T, int R, int MODE, bool F8 = false>
__global__ __launch_bounds__(RC_THREADS) void rowchain_kernel(NetDev net, RowArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using V = typename Op<T>::V;
  const LdsPlan P = lds_plan(net, R, (int)sizeof(T));
  T* const Xin = (T*)(smem + P.oXin);
  T* const GL = Xin;  // dL/drecon overwrites the input tile in place in the loss epilogue
  T* const P0b = (T*)(smem + P.oP0);
  T* const P1b = (T*)(smem + P.oP1);
  T* const Hc = (T*)(smem + P.oHc);
  T* const Q = Hc;  // condition-branch gradient overlays [h_traj ‖ h_c] (dead after fc fwd)
  T* const Dec = (T*)(smem + P.oDec);
  T* const Cin = (T*)(smem + P.oCin);
  float* const MuLv = (float*)(smem + P.oMuLv);
  float* const Dz = (float*)(smem + P.oDz);
  float* const Rch0 = (float*)(smem + P.oRch0);
  float* const Gd0 = (float*)(smem + P.oGd0);
  float* const Dhc2 = (float*)(smem + P.oU);
  float* const Start = (float*)(smem + P.oStart);
  int64_t* const RowG = (int64_t*)(smem + P.oRow);
  uint8_t* const Mask = (uint8_t*)(smem + P.oMask);
  float* const Part = (float*)(smem + P.oPart);
  float* const BiasL = (float*)(smem + P.oBias);
  uint8_t* const F8img = (uint8_t*)(smem + P.oF8);  // CVAE_FP8 only (0 B otherwise)
  // LDS buffer by id (a select chain on a uniform value: no runtime-indexed pointer array)
  T* const Cls = (T*)(smem + P.oCls);      // cfg4 only
  float* const Dce = (float*)(smem + P.oDce);
  auto buf = [&](int id) -> T* {
    return id == B_XIN ? Xin : id == B_P0 ? P0b : id == B_P1 ? P1b : id == B_HC ? Hc : id == B_DEC ? Dec
         : id == B_CLS ? Cls : Cin;
  };
  auto ld_of = [&](int id) -> int {
    return id == B_XIN ? P.sx : (id == B_P0 || id == B_P1) ? P.sp : id == B_HC ? P.shc : id == B_DEC ? P.sdec
         : id == B_CLS ? P.scls : P.scin;
  };

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int b0 = blockIdx.x * R;
  const int nrows = max(0, min(R, a.batch - b0));  // tiles past the batch write zeros
  const int Bp = net.Bp, Z = net.Z, H = net.H, S = net.S, D = net.D, I = net.I;
  const int mw = P.mw;
  const T* xg = (const T*)a.x;
  constexpr bool TRAIN = MODE == RC_TRAIN;
  const bool skip_cond = MODE == RC_DECODE && a.hc_in != nullptr;
  int stamp_i = 0;
  auto stamp = [&]() {
    if (CVAE_DIAG_STAMPS && a.stamps && tid == 0)
      gst<unsigned long long>(a.stamps + blockIdx.x * 64 + (stamp_i < 63 ? stamp_i : 63), __builtin_amdgcn_s_memrealtime());
    ++stamp_i;
  };

  float s_recon = 0.f, s_kl = 0.f, s_start = 0.f, s_t0 = 0.f, s_relu = 0.f;
  const uint64_t rng_off = rng_offset(a);
  const uint32_t erow0 = (uint32_t)a.eps_row0;

  // the weight stream starts before anything else: first block of the first step
  WBlock<T> pre;
  {
    const StepDesc s0 = a.steps[0];
    load_block(pre, (const T*)s0.W, s0.Kp & 0x3FFFFFFF, s0.Np, wave, 0);
  }
  // device counters: this launch begins optimizer step ctr[1] + 1 (the Adam kernel behind it reads
  // it and its scalars); one lane of block 0, while its wave waits for the first loads
  if (TRAIN && a.ctr && blockIdx.x == 0 && tid == 0) adam_precompute(a.ctr, a.lr, a.beta1, a.beta2, a.adam_pre);
  stamp();

  // ---------------------------------------------------------------- prologue: x tile, start points, LDS state
  auto zero = [&](void* p, int bytes) {
    f32x4* q = (f32x4*)p;
    for (int e = tid; e < bytes / 16; e += RC_THREADS) q[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto setup_lds = [&]() {  // step table, biases, zeroed concatenation buffers and masks
    for (int e = tid; e < a.nsteps * 4; e += RC_THREADS)
      ((u32x4*)(smem + P.oSteps))[e] = gld<u32x4>((const u32x4*)a.steps + e);
    for (int e = tid; e < net.nbias / 4 + 1; e += RC_THREADS)
      ((f32x4*)BiasL)[e] = e < net.nbias / 4 ? gld<f32x4>(net.bias_all + 4 * e) : f32x4{0.f, 0.f, 0.f, 0.f};
    zero(Hc, R * P.shc * (int)sizeof(T));
    zero(Dec, R * P.sdec * (int)sizeof(T));
    zero(Mask, rup(n_masks(net) * R * mw, 16));
    if (net.n_cls) {  // cfg4: the rows' one-hot class vectors (the class-embedding layer's input)
      for (int e = tid; e < R * P.scls; e += RC_THREADS) Cls[e] = to_t<T>(0.f);
    }
  };
  // after setup_lds and a barrier: set the one-hot entries (class of row r = classes[idx[b0+r]])
  auto set_classes = [&]() {
    if (!net.n_cls) return;
    for (int r = tid; r < nrows; r += RC_THREADS) {
      const int64_t g = a.idx ? gld<int64_t>(a.idx + b0 + r) : (int64_t)(b0 + r);
      int c = a.classes ? gld<int>(a.classes + g) : 0;
      c = c < 0 ? 0 : (c >= net.n_cls ? net.n_cls - 1 : c);  // out-of-range ids clamp (host validates)
      Cls[r * P.scls + c] = to_t<T>(1.f);
    }
  };
  // Fast path (absolute trajectories, 16-B aligned rows): task v = one 16-B vector of one row,
  // the 4 lanes of a quad holding the same vector of 4 consecutive rows.  Every lane loads its
  // vector and its row's first vector (the start point x[:,0,1:3], Training_VAE.py:345) at once
  // — no LDS round trip or barrier before the relative transform (:347-348) — writes the LDS
  // tile, and stores the feature-major arena copy of the tile as quad-transposed 8/16-B stores.
  constexpr int EPL = Op<T>::EPL, U = 5;
  const int VPR = I / EPL, NV = R * VPR;
  const bool vec = MODE != RC_DECODE && (I % EPL) == 0 && (((uintptr_t)xg) & 15) == 0 &&
                   (sizeof(T) == 4 || !a.x_f32);
  const bool fast = vec && !a.x_relative && NV <= U * RC_THREADS;
  if (fast) {
    const float inv_VPR = 1.f / (float)VPR, inv_Dd = 1.f / (float)D;
    const int last = max(a.batch - 1, 0);
    V xv[U], x0[U];
    int64_t gr[U];  // source row per task; rows past the batch re-read a valid row (zeroed below)
    int cc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = min(u * RC_THREADS + tid, NV - 1);
      const int w = v >> 2, rq = fdiv(w, inv_VPR), c = w - rq * VPR, row = 4 * rq + (v & 3);
      gr[u] = min(b0 + row, last);
      cc[u] = c;
    }
    if (a.idx) {  // all idx loads in flight together, then the x loads
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u * RC_THREADS < NV) gr[u] = gld<int64_t>(a.idx + gr[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u * RC_THREADS < NV) {  // wave-uniform
        xv[u] = gld<V>(xg + gr[u] * I + cc[u] * EPL);
        x0[u] = gld<V>(xg + gr[u] * I);
      }
    }
    setup_lds();  // overlaps the loads
    if (net.Ip > I) {
      for (int e = tid; e < R * (net.Ip - I); e += RC_THREADS) {
        const int r = e / (net.Ip - I), c = I + e % (net.Ip - I);
        Xin[r * P.sx + c] = to_t<T>(0.f);
      }
    }
    T* const xe0 = (T*)net.L[lE(net, 0)].xT;
    T* const xc0 = (T*)net.L[lC0(net)].xT;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = u * RC_THREADS + tid;
      if (u * RC_THREADS < NV && v < NV) {  // NV % 4 == 0: quads are whole
        const int w = v >> 2, rq = fdiv(w, inv_VPR), c = w - rq * VPR, row = 4 * rq + (v & 3);
        const bool live = row < nrows;
        const float s0 = live ? to_f(x0[u][1]) : 0.f, s1 = live ? to_f(x0[u][2]) : 0.f;
        const int f0 = c * EPL;
        int d = f0 - fdiv(f0, inv_Dd) * D;
        V o;
        float q[EPL];
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const float val = to_f(xv[u][e]) - (d == 1 ? s0 : 0.f) - (d == 2 ? s1 : 0.f);
          o[e] = to_t<T>(live ? val : 0.f);
          q[e] = to_f(o[e]);
          d = d + 1 == D ? 0 : d + 1;
        }
        *(V*)(Xin + row * P.sx + f0) = o;
        if (TRAIN) {
#pragma unroll
          for (int e = 0; e < EPL; e += 4)
            put4Tq(xe0, net.L[lE(net, 0)].Kp, f0 + e, b0 + row, f32x4{q[e], q[e + 1], q[e + 2], q[e + 3]});
        }
        if (c == 0) {  // quad-uniform: the condition input of this row (and its arena copy)
#pragma unroll
          for (int k = 0; k < 32; k += EPL) {
            V cv;
#pragma unroll
            for (int e = 0; e < EPL; ++e) cv[e] = to_t<T>(k + e == 0 ? s0 : k + e == 1 ? s1 : 0.f);
            *(V*)(Cin + row * P.scin + k) = cv;
          }
          if (TRAIN) put4Tq(xc0, net.L[lC0(net)].Kp, 0, b0 + row, f32x4{to_f(to_t<T>(s0)), to_f(to_t<T>(s1)), 0.f, 0.f});
        }
      }
    }
  } else {
    setup_lds();
    zero(Cin, R * P.scin * (int)sizeof(T));
    for (int r = tid; r < R; r += RC_THREADS) {
      float s0 = 0.f, s1 = 0.f;
      int64_t g = 0;
      if (r < nrows) {
        g = a.idx ? gld<int64_t>(a.idx + b0 + r) : (int64_t)(b0 + r);
        if (MODE == RC_DECODE || a.x_relative) {
          if (a.start_in) {  // decode(z, h_c) carries no start point
            s0 = gld<float>(a.start_in + (size_t)(b0 + r) * 2 + 0);
            s1 = gld<float>(a.start_in + (size_t)(b0 + r) * 2 + 1);
          }
        } else {
          // x[:,0,1:3]  (Training_VAE.py:345)
          s0 = a.x_f32 ? gld<float>((const float*)a.x + g * I + 1) : to_f(gld<T>(xg + g * I + 1));
          s1 = a.x_f32 ? gld<float>((const float*)a.x + g * I + 2) : to_f(gld<T>(xg + g * I + 2));
        }
      }
      Start[r * 2 + 0] = s0;
      Start[r * 2 + 1] = s1;
      RowG[r] = g;
    }
    lds_barrier();
    for (int r = tid; r < nrows; r += RC_THREADS) {
      Cin[r * P.scin + 0] = to_t<T>(Start[r * 2 + 0]);
      Cin[r * P.scin + 1] = to_t<T>(Start[r * 2 + 1]);
    }
    if (MODE != RC_DECODE) {
      for (int e = tid; e < R * net.Ip; e += RC_THREADS) {
        const int r = e / net.Ip, c = e - r * net.Ip;
        float v = 0.f;
        if (r < nrows && c < I) {
          const int d = c % D;
          v = a.x_f32 ? gld<float>((const float*)a.x + RowG[r] * I + c) : to_f(gld<T>(xg + RowG[r] * I + c));
          if (!a.x_relative) v -= (d == 1 ? Start[r * 2 + 0] : 0.f) + (d == 2 ? Start[r * 2 + 1] : 0.f);
        }
        Xin[r * P.sx + c] = to_t<T>(v);
      }
    } else {
      if (skip_cond) {
        for (int e = tid; e < R * H; e += RC_THREADS) {
          const int r = e / H, c = e - r * H;
          Dec[r * P.sdec + Z + c] = to_t<T>(r < nrows ? gld<float>(a.hc_in + (size_t)(b0 + r) * H + c) : 0.f);
        }
      }
      if (a.z_in) {
        for (int e = tid; e < R * Z; e += RC_THREADS) {
          const int r = e / Z, j = e - r * Z;
          Dec[r * P.sdec + j] = to_t<T>(r < nrows ? gld<float>(a.z_in + (size_t)(b0 + r) * Z + j) : 0.f);
        }
      }
    }
  }
  lds_barrier();
  stamp();

  // feature-major copy of input tiles for the weight-gradient kernel (one 4-row × 1-column quad
  // per task → one 8-B / 16-B store; the arena pads stay zero from creation)
  auto copy_T = [&](const T* src, int ld, int ncols, T* dst, int Kf) {
    constexpr int RQ = R / 4;
    for (int t = tid; t < ncols * RQ; t += RC_THREADS) {
      const int c = t / RQ, q = t - c * RQ;
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = to_f(src[(4 * q + i) * ld + c]);
      gstore4(dst + aoff(c, b0 + 4 * q, Kf), v);
    }
  };
  // slow path only: the condition and x tiles (the fast path stored them from its prologue)
  if (TRAIN && !fast && !CVAE_DIAG_NOSTORE) {
    copy_T(Cin, P.scin, 2, (T*)net.L[lC0(net)].xT, net.L[lC0(net)].Kp);
    copy_T(Xin, P.sx, I, (T*)net.L[lE(net, 0)].xT, net.L[lE(net, 0)].Kp);
  }
  if (net.n_cls) {  // cfg4: the one-hot class input of the class-embedding step
    set_classes();
    lds_barrier();
    if (TRAIN && !CVAE_DIAG_NOSTORE) copy_T(Cls, P.scls, net.n_cls, (T*)net.L[lCE(net)].xT, net.L[lCE(net)].Kp);
  }

  const float Bf = (float)a.batch;
  const float inv_BSD = 1.f / (Bf * (float)(S * D));
  const float inv_2B = 1.f / (2.f * Bf);
  const float inv_B = 1.f / Bf;
  const float inv_BS1 = S > 1 ? 1.f / (Bf * (float)(S - 1)) : 0.f;
  const float inv_BZ = 1.f / (Bf * (float)Z);
  // Training_VAE.py:247, :256; the external-gradient backward takes dL/drecon as given
  const bool use_start = !a.ext && a.w_start > 0.f, use_time = !a.ext && a.w_time > 0.f;
  const bool prim = R >= 16 || (lane & 15) < R;  // this lane's row is not a duplicate (R < 16)
  const float inv_D = 1.f / (float)D, inv_S = 1.f / (float)S, inv_Z = 1.f / (float)Z;
  const float inv_Zp2 = 1.f / (float)net.Zp2;
  const uint8_t* mkEl = Mask + (2 + net.n_enc - 1) * R * mw;  // last encoder layer
  const uint8_t* mkC1 = Mask + 1 * R * mw;

  // ---------------------------------------------------------------- the step interpreter
  const StepDesc* const StepsL = (const StepDesc*)(smem + P.oSteps);
  auto sgpr = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); };
  auto sptr = [&](uint32_t lo, uint32_t hi) { return (void*)(((uint64_t)sgpr(hi) << 32) | sgpr(lo)); };
  for (int si = 0; si < a.nsteps; ++si) {
    // this step's descriptor and the next step's weight operand, from LDS, made scalar
    const u32x4* dq = (const u32x4*)(StepsL + si);
    const u32x4 q0 = dq[0], q1 = dq[1], q2 = dq[2], q3 = dq[3];
    const bool has_next = si + 1 < a.nsteps;
    const u32x4* nq = (const u32x4*)(StepsL + (has_next ? si + 1 : si));
    const u32x4 n0 = nq[0], n1 = nq[1];
    const T* const W = (const T*)sptr(q0.x, q0.y);
    T* const g1 = (T*)sptr(q0.z, q0.w);
    T* const g2 = (T*)sptr(q1.x, q1.y);
    const uint32_t kraw = sgpr(q1.z);
    const bool f8 = F8 && ((kraw >> 30) & 1);  // CVAE_FP8 forward step (Kp then counts K/2: the e4m3 pair chunks)
    const int Kp = (int)(kraw & 0x3FFFFFFFu), Np = (int)sgpr(q1.w), N = (int)sgpr(q2.x), bias_off = (int)sgpr(q2.y);
    const uint32_t code = sgpr(q2.z);
    const int off1 = (int)sgpr(q2.w), off2 = (int)sgpr(q3.x);
    const uint32_t goff = sgpr(q3.y);
    const int kf1 = (int)sgpr(q3.z), kf2 = (int)sgpr(q3.w);
    const int goff1 = (int)(goff & 0xFFFF), goff2 = (int)(goff >> 16);
    const T* const nW = has_next ? (const T*)sptr(n0.x, n0.y) : (const T*)nullptr;
    const int nKp = (int)(sgpr(n1.z) & 0x3FFFFFFFu), nNp = (int)sgpr(n1.w);
    const int xbuf = code & 15, kind = (code >> 4) & 15;
    const int dst1 = (int)((code >> 8) & 15) - 1, dst2 = (int)((code >> 12) & 15) - 1;
    const bool concat = (code >> 16) & 1, hc_o = (code >> 17) & 1, linear = (code >> 18) & 1;
    const int mask_out = (int)((code >> 20) & 63) - 1, mask_in = (int)((code >> 26) & 63) - 1;
    T* const d1 = dst1 >= 0 ? buf(dst1) : nullptr;
    T* const d2 = dst2 >= 0 ? buf(dst2) : nullptr;
    const int ld1 = dst1 >= 0 ? ld_of(dst1) : 0;
    const int ld2 = dst2 >= 0 ? ld_of(dst2) : 0;
    uint8_t* const mko = Mask + (mask_out >= 0 ? mask_out : 0) * R * mw;
    const uint8_t* const mki = Mask + (mask_in >= 0 ? mask_in : 0) * R * mw;

#if CVAE_DIAG_SUB
    g_sub_step = si;
    SUBSTAMP(0);
#endif
    // the step's bias lives in LDS (copied once in the prologue): the epilogue issues no
    // global loads, so it never waits behind the weight prefetch (vmcnt retires in order)
    const float* const biasL = BiasL + (bias_off >= 0 ? bias_off : net.nbias);
    // CVAE_FP8 wide step: its input converted once into the e4m3 image (F8_IMG_K above)
    const bool f8img = F8 && f8 && 2 * Kp <= F8_IMG_K;
    if constexpr (Op<T>::EPL == 8) {
      if (f8img) {
        const T* const X8 = buf(xbuf);
        const int ldx8 = ld_of(xbuf), nch = 2 * Kp / 32;
        for (int it = threadIdx.x; it < R * nch * 4; it += RC_THREADS) {
          const int q = it & 3, rc = it >> 2, r = rc / nch, c = rc - r * nch;
          *(long*)(F8img + r * F8_LD + c * 32 + q * 8) = f8x8(xchunk<T>(X8 + r * ldx8 + c * 32, q));
        }
        lds_barrier();
      }
    }

    // One dense instance per epilogue kind (the switch is wave-uniform): each epilogue compiles
    // straight-line with only its own live values.
    auto run = [&](auto&& epi) {
      dense<T, R, true>(buf(xbuf), ld_of(xbuf), W, Kp, Np, pre, nW, nKp, nNp, biasL, epi, f8,
                        f8 ? f8_header(W)->inv_s : 1.f, f8img ? F8img : nullptr);
    };
    auto run_nb = [&](auto&& epi) {  // backward steps: no bias
      dense<T, R, false>(buf(xbuf), ld_of(xbuf), W, Kp, Np, pre, nW, nKp, nNp, biasL, epi);
    };
    // forward hidden layer: ReLU, mask nibble, LDS dst(s), arena xT of consumers
    auto epi_relu = [&](int row, int f0, f32x4 v, f32x4 b4) {
      if (CVAE_DIAG_NOEPI) return;
      const bool live = row < nrows;
      f32x4 y;
      uint32_t nib = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float u = v[i] + b4[i];
        y[i] = live ? (linear ? u : fmaxf(u, 0.f)) : 0.f;  // zero-padded bias: pad features come out 0
        nib |= (y[i] > 0.f ? 1u : 0u) << i;
      }
      // this lane owns (row, f0..f0+3): no atomics; the class-embedding step (linear) has no mask
      if (!CVAE_DIAG_NOLDSW && !linear) mko[row * mw + (f0 >> 2)] = (uint8_t)nib;
      if (concat && f0 >= N) return;  // part of a concatenation: never write its pads
      if (!CVAE_DIAG_NOLDSW) put4(d1 + row * ld1 + off1 + f0, y);
      if (d2 && !CVAE_DIAG_NOLDSW) put4(d2 + row * ld2 + off2 + f0, y);
      if (g1) put4Tq(g1, kf1, goff1 + f0, b0 + row, y);
      if (g2) put4Tq(g2, kf2, goff2 + f0, b0 + row, y);
      if (!TRAIN && hc_o && a.hc_out && live && f0 < N) gst<f32x4>(a.hc_out + (size_t)(b0 + row) * H + f0, y);
    };
    // backward: mask with the producer's ReLU bits
    auto epi_bwd = [&](int row, int f0, f32x4 v, f32x4) {
      if (CVAE_DIAG_NOEPI) return;
      const uint32_t nib = mask4(mki, mw, row, f0);
      f32x4 y;
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = (nib >> i) & 1u ? v[i] : 0.f;
      if (d1) put4(d1 + row * ld1 + f0, y);
      put4Tq(g1, kf1, f0, b0 + row, y);
    };
    // mu ‖ logvar, fp32 in LDS
    auto epi_fc = [&](int row, int f0, f32x4 v, f32x4 b4) {
      if (CVAE_DIAG_NOEPI) return;
      const bool live = row < nrows;
      f32x4 y;
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = live ? v[i] + b4[i] : 0.f;
      *(f32x4*)(MuLv + row * net.Zp2 + f0) = y;
      if (MODE == RC_FWD && live) {  // Z % 4 == 0: a 4-feature group is all mu or all logvar
        if (f0 < Z) {
          if (a.mu_out) gst<f32x4>(a.mu_out + (size_t)(b0 + row) * Z + f0, y);
        } else if (f0 < 2 * Z && a.lv_out) {
          gst<f32x4>(a.lv_out + (size_t)(b0 + row) * Z + f0 - Z, y);
        }
      }
    };
    // recon r = acc + bias (fp32); dL/dr → GL (LDS) + gT
    auto epi_loss = [&](int row, int f0, f32x4 v, f32x4 b4) {
      if (CVAE_DIAG_NOEPI) return;
      const bool live = row < nrows;
      f32x4 y;
      // target x_rel from the resident input tile; GL overwrites it in place below
      // (same lane, same elements), so no other reader is affected
      const f32x4 xr = get4(Xin + row * P.sx + f0);
      int s = fdiv(f0, inv_D), d = f0 - s * D;

#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float gi = 0.f;
        if (live && f0 + i < I && a.ext) {  // cvae_backward: dL/drecon given
          gi = a.d_recon ? gld<float>(a.d_recon + (size_t)(b0 + row) * I + f0 + i) : 0.f;
          if (d == 0) Gd0[row * S + s] = gi;
        } else if (live && f0 + i < I) {
          const float r = v[i] + b4[i];
          const float diff = r - xr[i];
          s_recon += prim ? diff * diff : 0.f;
          gi = a.w_recon * 2.f * diff * inv_BSD;
          if (s == 0 && (d == 1 || d == 2) && use_start) {
            s_start += prim ? diff * diff : 0.f;
            gi += a.w_start * 2.f * diff * inv_2B;
          }
          if (d == 0) {
            Rch0[row * S + s] = r;
            if (s == 0 && use_time) {
              s_t0 += prim ? r * r : 0.f;
              gi += a.w_time * 2.f * r * inv_B;
            }
            Gd0[row * S + s] = gi;
          }
        }
        y[i] = gi;
        // the time channel (d == 0) is finished by the fix-up pass once its neighbours exist
        if (!CVAE_DIAG_NOSTORE && (d != 0 || f0 + i >= I)) gst<T>(g1 + aoff(f0 + i, b0 + row, kf1), to_t<T>(gi));
        if (++d == D) { d = 0; ++s; }
      }
      put4(GL + row * P.sx + f0, y);  // d == 0 entries are overwritten by the fix-up pass
    };
    auto epi_recon = [&](int row, int f0, f32x4 v, f32x4 b4) {
      if (CVAE_DIAG_NOEPI) return;
      if (!a.recon_out || row >= nrows) return;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (f0 + i < I) gst<float>(a.recon_out + (size_t)(b0 + row) * I + f0 + i, v[i] + b4[i]);
    };
    // decoder L0 backward: dz and the decoder's share of dh_c (Z, H multiples of 4: no straddle)
    auto epi_d0b = [&](int row, int f0, f32x4 v, f32x4) {
      if (CVAE_DIAG_NOEPI) return;
      if (f0 < Z) {
        *(f32x4*)(Dz + row * Z + f0) = v;
      } else if (f0 < Z + H) {
        f32x4 y = v;
        if (a.ext && a.d_hc && row < nrows) y += gld<f32x4>(a.d_hc + (size_t)(b0 + row) * H + f0 - Z);  // H % 4 == 0
        *(f32x4*)(Dhc2 + row * H + f0 - Z) = y;
      } else if (f0 < Z + H + net.cls_dim) {  // cfg4: the decoder's share of de (cls_dim % 4 == 0)
        *(f32x4*)(Dce + row * net.cls_dim + f0 - Z - H) = v;
      }
    };
    // dh = G_fc·W_fc → [dh_traj ‖ dh_c(fc share)]   (H % 4 == 0: no straddle)
    auto epi_fcb = [&](int row, int f0, f32x4 v, f32x4) {
      if (CVAE_DIAG_NOEPI) return;
      f32x4 y;
      if (f0 < H) {
        const uint32_t nib = mask4(mkEl, mw, row, f0);
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = (nib >> i) & 1u ? v[i] : 0.f;
        put4(P1b + row * P.sp + f0, y);
        put4Tq(g1, kf1, f0, b0 + row, y);
      } else if (f0 < 2 * H) {
        const int c = f0 - H;
        const uint32_t nib = mask4(mkC1, mw, row, c);
        const f32x4 dh2 = *(const f32x4*)(Dhc2 + row * H + c);
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = (nib >> i) & 1u ? v[i] + dh2[i] : 0.f;
        put4(Q + row * P.shc + c, y);
        put4Tq(g2, kf2, c, b0 + row, y);
      } else if (f0 < 2 * H + net.cls_dim) {  // cfg4: de = fc share + decoder share (no activation)
        const int c = f0 - 2 * H;
        const f32x4 y2 = v + *(const f32x4*)(Dce + row * net.cls_dim + c);
        const LayerDev& LC = net.L[lCE(net)];
        put4Tq((T*)LC.gT, LC.Np, c, b0 + row, y2);
      }
    };
    switch (kind) {
      case E_RELU: run(epi_relu); break;
      case E_FC: if constexpr (MODE != RC_DECODE) run(epi_fc); break;
      case E_LOSS: if constexpr (TRAIN) run(epi_loss); break;
      case E_RECON: if constexpr (!TRAIN) run(epi_recon); break;
      case E_BWD: if constexpr (TRAIN) run_nb(epi_bwd); break;
      case E_D0B: if constexpr (TRAIN) run_nb(epi_d0b); break;
      default: if constexpr (TRAIN) run_nb(epi_fcb); break;
    }
    lds_barrier();
#if CVAE_DIAG_SUB
    SUBSTAMP(4);
#endif

    // ------------------------------------------------------------ element-wise phases after a step
    if (kind == E_FC && MODE != RC_DECODE) {
      // reparameterize (:199-206) + KL terms (:243)
      T* xd0 = (T*)net.L[lD(net, 0)].xT;
      for (int e = tid; e < R * Z; e += RC_THREADS) {
        const int r = fdiv(e, inv_Z), j = e - r * Z;
        float z = 0.f, ep = 0.f, sd = 0.f;
        if (r < nrows) {
          const float mu = MuLv[r * net.Zp2 + j], lv = MuLv[r * net.Zp2 + Z + j];
          sd = expf(0.5f * lv);
          ep = a.eps ? gld<float>(a.eps + (size_t)(b0 + r) * Z + j)
                     : philox_normal(a.seed, rng_off, erow0 + (uint32_t)(b0 + r), (uint32_t)j);
          z = mu + ep * sd;
          s_kl += 1.f + lv - mu * mu - expf(lv);
          if (MODE == RC_FWD && a.eps_out) gst<float>(a.eps_out + (size_t)(b0 + r) * Z + j, ep);
        }
        Dec[r * P.sdec + j] = to_t<T>(z);
        if (TRAIN && !CVAE_DIAG_NOSTORE) gst<T>(xd0 + aoff(j, b0 + r, net.L[lD(net, 0)].Kp), to_t<T>(z));
      }
      lds_barrier();
    } else if (kind == E_LOSS) {
      // time-monotonicity term: relu(r_s - r_{s+1}) (:261-262), ReLU'(0) = 0
      T* gl = g1;
      for (int e = tid; e < R * S; e += RC_THREADS) {
        const int r = fdiv(e, inv_S), s = e - r * S;
        float g = 0.f;
        if (r < nrows) {
          g = Gd0[r * S + s];
          if (use_time) {
            if (s < S - 1) {
              const float u = Rch0[r * S + s] - Rch0[r * S + s + 1];
              if (u > 0.f) {
                g += a.w_time * inv_BS1;
                s_relu += u;
              }
            }
            if (s > 0) {
              const float u = Rch0[r * S + s - 1] - Rch0[r * S + s];
              if (u > 0.f) g -= a.w_time * inv_BS1;
            }
          }
        }
        GL[r * P.sx + s * D] = to_t<T>(g);
        if (!CVAE_DIAG_NOSTORE) gst<T>(gl + aoff(s * D, b0 + r, kf1), to_t<T>(g));
      }
      lds_barrier();
    } else if (kind == E_D0B) {
      // reparameterisation + KL backward → G_fc = [dmu ‖ dlogvar] into P0 (the fc-backward input)
      T* gfc = (T*)net.L[lFC(net)].gT;
      for (int e = tid; e < R * net.Zp2; e += RC_THREADS) {
        const int r = fdiv(e, inv_Zp2), c = e - r * net.Zp2;
        float g = 0.f;
        if (r < nrows && c < 2 * Z) {
          const int j = c < Z ? c : c - Z;
          const float dz = Dz[r * Z + j];
          if (a.ext) {  // cvae_backward: dL/dmu, dL/dlogvar given (+ the reparameterisation path)
            const float gin = c < Z ? (a.d_mu ? gld<float>(a.d_mu + (size_t)(b0 + r) * Z + j) : 0.f)
                                    : (a.d_lv ? gld<float>(a.d_lv + (size_t)(b0 + r) * Z + j) : 0.f);
            if (c < Z) {
              g = gin + dz;
            } else {
              const float lv = MuLv[r * net.Zp2 + Z + j];
              const float sd = expf(0.5f * lv);
              const float ep = a.eps ? gld<float>(a.eps + (size_t)(b0 + r) * Z + j)
                                     : philox_normal(a.seed, rng_off, erow0 + (uint32_t)(b0 + r), (uint32_t)j);
              g = gin + dz * ep * 0.5f * sd;
            }
          } else if (c < Z) {
            g = a.w_kld * MuLv[r * net.Zp2 + j] * inv_BZ + dz;
          } else {
            // eps and std are recomputed (same draw, same expf) rather than kept in LDS: at
            // latent 512 two R x Z fp32 buffers would not fit beside the rest of the tile state
            const float lv = MuLv[r * net.Zp2 + Z + j];
            const float sd = expf(0.5f * lv);
            const float ep = a.eps ? gld<float>(a.eps + (size_t)(b0 + r) * Z + j)
                                   : philox_normal(a.seed, rng_off, erow0 + (uint32_t)(b0 + r), (uint32_t)j);
            g = a.w_kld * 0.5f * (expf(lv) - 1.f) * inv_BZ + dz * ep * 0.5f * sd;
          }
        }
        P0b[r * P.sp + c] = to_t<T>(g);
        if (!CVAE_DIAG_NOSTORE) gst<T>(gfc + aoff(c, b0 + r, net.L[lFC(net)].Np), to_t<T>(g));
      }
      // pads of the two gradient targets of the fc backward must read as zero
      if (net.Hp > H) {
        for (int e = tid; e < R * (net.Hp - H); e += RC_THREADS) {
          const int r = e / (net.Hp - H), c = H + e % (net.Hp - H);
          P1b[r * P.sp + c] = to_t<T>(0.f);
          Q[r * P.shc + c] = to_t<T>(0.f);
        }
      }
      lds_barrier();
    }
    stamp();
  }
  if (!TRAIN) return;

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
  lds_barrier();
  if (tid < 5) {
    float s = 0.f;
    for (int w = 0; w < RC_NW; ++w) s += Part[w * 8 + tid];
    gst<float>(a.partials + blockIdx.x * 8 + tid, s);
  }
}
