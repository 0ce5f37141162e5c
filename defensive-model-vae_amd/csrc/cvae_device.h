// cvae_device.h — device-side data structures and CDNA4 building blocks for the
// conditional trajectory VAE hot path (gfx950 only).
//
// Layout conventions:
//  * Every Linear layer l has padded dims Kp = roundup(in, 32), Np = roundup(out, 32).
//  * Device weight copies in the operand dtype T (fp32 or bf16), in MFMA fragment order
//    (frag_off below):
//      Wf ~ [Np][Kp]  (= nn.Linear (out,in) zero-padded) — operand of the forward GEMM
//      Wb ~ [Kp][Np]  (= Wᵀ zero-padded)                  — operand of the dX GEMM
//    plus a padded fp32 bias[Np].  The fp32 master parameters stay in the
//    caller's flat state_dict-ordered buffer.
//  * Activation arena, TILE-MAJOR feature-major in T: a matrix with Kf feature rows (Kf = Kp for
//    xT, Np for gT) is [Bp/16 row tiles][Kf features][16 batch rows] (aoff below):
//      xT(l) = input of layer l, gT(l) = dL/d(pre-activation) of layer l.
//    A row-chain workgroup (16 batch rows) writes one contiguous [Kf][16] slab, so its epilogue
//    stores are whole 512-B runs; the weight-gradient kernel reduces over the batch with both
//    operands batch-contiguous in 16-row runs: dW_l = gT(l) · xT(l)ᵀ.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CVAE_MAX_LAYERS 40
#define CVAE_NW 4            // waves per workgroup
#define CVAE_THREADS 256

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

struct LayerDev {
  int K, N, Kp, Np;      // real / padded in-out dims
  int relu;              // 1: ReLU after this layer
  int nseg, seg_rows0;   // parameter segments along N (fc fuses mu‖logvar: 2 segments)
  int f8;                // CVAE_FP8: Wf holds OCP e4m3 fragments (pair-chunk order, f8_wf_off), see below
  int wt;                // master weight stored [K][N] (nn.Embedding layout: the class-embedding layer)
  int has_bias;          // 0: no bias parameter (the class-embedding layer); its padded bias stays 0
  int f8b;               // CVAE_FP8: Wb8 holds e4m3(s·Wᵀ) K-pair fragments for an e4m3 dX GEMM (the wide chain)
  int64_t pw[2], pb[2];  // flat fp32 offsets of weight / bias of each segment
  void* Wf;              // [Np][Kp] T  (f8: [Np][Kp] e4m3, preceded by the F8Scale header)
  void* Wb;              // [Kp][Np] T
  void* Wb8;             // f8b: [Kp][Np] e4m3, pair-chunk order (f8_wf_off over K = Np); the scale is Wf's
  float* bias;           // [Np] fp32
  void* xT;              // [Kp][Bp] T   input of the layer (feature-major)
  void* gT;              // [Np][Bp] T   gradient w.r.t. pre-activation
};

struct NetDev {
  int S, D, Z, H, I;
  int n_enc, n_dec, n_layers;
  int Ip, Hp, Hcp, ZHp, Zp2, Cp;
  int n_cls, cls_dim, Clsp;  // BASELINE cfg4 class embedding (0 = the reference model); Clsp = rup(n_cls, 32)
  int Bp;                // arena row capacity
  int dtype;             // 0 fp32, 1 bf16
  const float* zbias;    // zeros (>= max Np floats): the "bias" of the dX GEMMs
  const float* bias_all; // every layer's padded bias back to back (LayerDev::bias points into it)
  int nbias;             // floats in bias_all (a multiple of 32)
  int bias_off[CVAE_MAX_LAYERS];
  LayerDev L[CVAE_MAX_LAYERS];
};

// layer indices: C0=0, C1=1, E0=2 .. E0+n_enc-1, FC, D0 .. D0+n_dec-1
__host__ __device__ inline int lC0(const NetDev&) { return 0; }
__host__ __device__ inline int lC1(const NetDev&) { return 1; }
__host__ __device__ inline int lE(const NetDev&, int i) { return 2 + i; }
__host__ __device__ inline int lFC(const NetDev& n) { return 2 + n.n_enc; }
__host__ __device__ inline int lD(const NetDev& n, int i) { return 3 + n.n_enc + i; }
// class-embedding layer (cfg4): one-hot(class) → e, after the decoder (its table is the last
// parameter tensor, so the reference's 24 keys and init order come first)
__host__ __device__ inline int lCE(const NetDev& n) { return 3 + n.n_enc + n.n_dec; }

// ni: input tiles per workgroup of the generic dW kernel (0/1: 32 × 32, 2: 32 × 64; wgrad_kernel)
struct TileDesc { int layer, o0, i0, ni; };

// element (feature f, batch row b) of an arena matrix with Kf feature rows
__host__ __device__ inline size_t aoff(int f, int b, int Kf) {
  return ((size_t)(b >> 4) * Kf + f) * 16 + (b & 15);
}

// ------------------------------------------------------------------ operand types
template <typename T> struct Op;
template <> struct Op<float> {
  using V = f32x4;            // 16 B per lane = 4 fp32 along K
  static constexpr int EPL = 4;
  static constexpr int KC = 16;   // K covered by one 16-B fragment (4 MFMA 16x16x4)
};
template <> struct Op<__bf16> {
  using V = bf16x8;           // 16 B per lane = 8 bf16 along K
  static constexpr int EPL = 8;
  static constexpr int KC = 32;   // one MFMA 16x16x32
};

// acc += A·B over one 16-B-per-lane K chunk.  Lane l holds A[l&15][kq..kq+EPL) and
// B[kq..kq+EPL)[l&15], kq = EPL*(l>>4).  For fp32 the four 16x16x4 MFMAs take element j
// of every lane, i.e. a permuted but identical K order on both operands.
__device__ __forceinline__ f32x4 mfma_chunk(f32x4 a, f32x4 b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  return c;
}
__device__ __forceinline__ f32x4 mfma_chunk(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Operand copies (Wf, Wb) are stored in MFMA FRAGMENT ORDER: for n-tile t (16 output rows) and
// K chunk kc, the 64 lanes' 16-B fragments are contiguous — 1 KB per (t, kc) — so one wave load
// instruction reads 8 full 128-B lines.  (Row-major [Np][Kp] makes each instruction 16 rows x
// 64 B: texture-address bound at ~38 GB/s per CU, measured 3.7x slower — scripts/ubench/wload.hip.)
// Lane (r, q) of a fragment holds row 16t + r and the chunk-relative K positions frag_k(q, e):
//   bf16: 4q + e for e < 4, 16 + 4q + (e - 4) for e >= 4 — the K order two transposed LDS block
//         reads of a feature-major activation image deliver (ds_read_b64_tr_b16, cvae_fastchain.h);
//         the MFMA sums over all 32 positions, so any order works as long as A and B agree;
//   fp32: 4q + e.
template <typename T>
__host__ __device__ inline int frag_k(int q, int e) {
  return Op<T>::EPL == 8 ? (e < 4 ? 4 * q + e : 12 + 4 * q + e) : 4 * q + e;
}
// Element (n, k) of an operand matrix with padded K extent Kp:
template <typename T>
__host__ __device__ inline size_t frag_off(int n, int k, int Kp) {
  constexpr int EPL = Op<T>::EPL, KC = Op<T>::KC;
  const int t = n >> 4, r = n & 15, kc = k / KC, kk = k - kc * KC;
  const int q = EPL == 8 ? (kk & 15) >> 2 : kk >> 2;
  const int e = EPL == 8 ? (kk & 3) + ((kk >> 4) << 2) : kk & 3;
  return ((size_t)(t * (Kp / KC) + kc) * 64 + q * 16 + r) * EPL + e;
}

// ------------------------------------------------------------------ fp8 forward operands (CVAE_FP8)
// BASELINE cfg5 asks for fp8 MFMA GEMMs.  With dtype CVAE_FP8 every forward layer whose padded K
// is a multiple of 64 multiplies OCP e4m3 weights by e4m3 activations (v_mfma_f32_16x16x32_fp8_fp8,
// fp32 accumulate); activations, arena, dX (Wb) and dW stay bf16, master weights/Adam/loss fp32.
// Weights carry a per-layer power-of-two scale s (F8Scale, written on the device by
// cvae_pack_weights from the layer's |W| max with 4x headroom): Wf = e4m3(s·W), and the
// forward epilogue multiplies the accumulator by 1/s.  Activations are converted unscaled
// (saturating at ±448).  Layout: a 16-B lane fragment holds TWO 32-wide K chunks (2c in bytes
// 0-7, 2c+1 in bytes 8-15), each in frag_k order — so a step loads 16 B per (n-tile, K/64
// pair) exactly like a bf16 step over half the K: the weight stream halves.
struct F8Scale { float s, inv_s; float pad_[62]; };  // 256 B in front of Wf
constexpr float F8_MAX = 448.f;
__host__ __device__ inline size_t f8_wf_off(int n, int kc, int Kp) {  // byte offset of lane-fragment (n-tile, chunk kc) lane 0
  return ((size_t)((n >> 4) * (Kp / 64) + (kc >> 1)) * 64) * 16 + (kc & 1) * 8;
}
__device__ __forceinline__ const F8Scale* f8_header(const void* Wf) {
  return (const F8Scale*)((const char*)Wf - sizeof(F8Scale));
}
// ---- MX (block-scaled e4m3) operands of v_mfma_scale_f32_16x16x128_f8f6f4 (the wide chain's dX
// GEMMs, cvae_widechain.h gemm_mxb; the MX dW, cvae_wgrad.h mx_dw_chunk).  A lane's 32 bytes are
// four 8-byte quarters h; the instruction's MX block b of row r is quarters 2(b >> 1), 2(b >> 1) + 1
// of the lanes r + 16j with j >> 1 == b & 1 (mapped on the GPU: scripts/ubench/mxscale.hip), and its
// E8M0 scale comes from lane r + 16b.
typedef long l2 __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
// saturation to ±448 before an e4m3 conversion: one v_med3_f32 (fminf(fmaxf(..)) compiled to a
// canonicalizing v_max_f32 plus the same med3: two VALU per value; equal for every non-NaN input)
__device__ __forceinline__ float f8_sat(float x) { return __builtin_amdgcn_fmed3f(x, -F8_MAX, F8_MAX); }
// 8 values → 8 e4m3 bytes (RNE, saturated to ±448), element e in byte e
__device__ __forceinline__ long f8x8(const float (&v)[8]) {
  int w0 = 0, w1 = 0;
  auto c = [](float x) { return f8_sat(x); };
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c(v[0]), c(v[1]), w0, false);
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c(v[2]), c(v[3]), w0, true);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c(v[4]), c(v[5]), w1, false);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c(v[6]), c(v[7]), w1, true);
  return (long)(unsigned)w0 | ((long)(unsigned)w1 << 32);
}
__device__ __forceinline__ long f8x8(bf16x8 x) {
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
  return f8x8(v);
}

template <typename T> __device__ __forceinline__ T to_t(float v);
template <> __device__ __forceinline__ float to_t<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 to_t<__bf16>(float v) { return (__bf16)v; }
__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(__bf16 v) { return (float)v; }

// store 4 consecutive T values (8 B for bf16, 16 B for fp32)
__device__ __forceinline__ void store4(float* p, f32x4 v) { *(f32x4*)p = v; }
__device__ __forceinline__ void store4(__bf16* p, f32x4 v) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 h;
  h[0] = (__bf16)v[0]; h[1] = (__bf16)v[1]; h[2] = (__bf16)v[2]; h[3] = (__bf16)v[3];
  *(bf16x4*)p = h;
}

// ------------------------------------------------------------------ global-address-space access
// Pointers that come out of descriptors in memory are generic: hipcc then emits FLAT
// loads/stores, which count on lgkmcnt as well as vmcnt — every LDS wait would also wait for
// the in-flight weight stream and arena stores.  These casts force global_* instructions.
#define CVAE_GLOBAL __attribute__((address_space(1)))
template <typename V>
__device__ __forceinline__ V gld(const void* p) { return *(const CVAE_GLOBAL V*)p; }
template <typename V>
__device__ __forceinline__ void gst(void* p, V v) { *(CVAE_GLOBAL V*)p = v; }

// Store of the dW ⊕ Adam epilogue (master state, operand copies).  CVAE_WT_STORES=1 makes it a
// write-through buffer store (sc1 cache policy = aux 16 on gfx950: the line leaves the XCD's L2 now
// instead of in the kernel-end writeback) — measured slower (dW 8.2-8.3 vs 7.7-7.9 µs, round 3,
// profiles/r03d), so the default is the plain global store.  `base` must be wave-uniform (it
// becomes the buffer resource); the byte offset is per lane and below 2^31.
#ifndef CVAE_WT_STORES
#define CVAE_WT_STORES 0
#endif
template <typename V>
__device__ __forceinline__ void st_wt(void* base, size_t byte_off, V v) {
  if (!CVAE_WT_STORES) {
    gst<V>((char*)base + byte_off, v);
    return;
  }
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  static_assert(sizeof(V) == 16 || sizeof(V) == 8 || sizeof(V) == 4, "16, 8 or 4 bytes");
  typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
  if constexpr (sizeof(V) == 16)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)byte_off, 0, 16);
  else if constexpr (sizeof(V) == 8)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, (int)byte_off, 0, 16);
  else
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)byte_off, 0, 16);
}

// ------------------------------------------------------------------ Adam step scalars (device step counters)
// torch's two per-step Adam scalars from the step count t, in doubles as Python forms them
// (torch/optim/adam.py: bias_correction1 = 1 - beta1 ** step, step_size = lr / bias_correction1,
// bias_correction2_sqrt = bias_correction2 ** 0.5), rounded to fp32 where the tensor op takes them
__device__ __forceinline__ void adam_scalars(double lr, double b1, double b2, double t, float& lr_neg_step,
                                             float& bc2_sqrt) {
  const double bc1 = 1.0 - pow(b1, t);
  const double bc2 = 1.0 - pow(b2, t);
  lr_neg_step = (float)(-(lr / bc1));
  bc2_sqrt = (float)sqrt(bc2);
}
typedef float adam_f32x2 __attribute__((ext_vector_type(2)));
// one lane, at the start of a training step: ctr[1] += 1 and the scalars of that step into ctr[2]
__device__ __forceinline__ void adam_precompute(uint64_t* ctr, double lr, double b1, double b2, bool scalars) {
  const uint64_t t = ctr[1] + 1;
  ctr[1] = t;
  if (scalars) {
    float a, b;
    adam_scalars(lr, b1, b2, (double)t, a, b);
    *(adam_f32x2*)(ctr + 2) = adam_f32x2{a, b};
  }
}

// ------------------------------------------------------------------ Philox4x32-10
#ifndef CVAE_DIAG_PHILOX_ROUNDS
#define CVAE_DIAG_PHILOX_ROUNDS 10  // diagnostic builds only (A/B of the draw's cost)
#endif
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < CVAE_DIAG_PHILOX_ROUNDS; ++i) {
    // one 32 x 32 -> 64-bit product per word (v_mad_u64_u32) instead of separate lo and hi multiplies
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// Box-Muller on one pair of Philox words: (rad·cos, rad·sin) with rad = sqrt(-2 ln f0), f0 in
// (0, 1], and the angle 2π·f1, f1 in [0, 1).  The bare hardware instructions: v_log_f32 (log2;
// f0 >= 2^-32 is normal, so no denormal scaling), v_sqrt_f32, and v_sin_f32 / v_cos_f32, which
// take the angle in revolutions (f1 itself).  Each is ~1 ulp, and eps is a random draw.  sqrtf,
// __logf and __sinf wrap these in a correctly rounded sqrt, an extended-precision ln and a 1/(2π)
// multiply: ~40 instead of 12 VALU per pair.
__device__ __forceinline__ void box_muller(uint32_t u0, uint32_t u1, float& c, float& s) {
  const float f0 = ((float)u0 + 1.0f) * 2.3283064365386963e-10f;  // (0,1]
  const float f1 = (float)u1 * 2.3283064365386963e-10f;
  const float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(f0));  // -2 ln 2 · log2
  c = rad * __builtin_amdgcn_cosf(f1);
  s = rad * __builtin_amdgcn_sinf(f1);
}

// standard normal eps for (row b, latent j): Box-Muller on Philox(seed; b, j/4, offset)
__device__ __forceinline__ float philox_normal(uint64_t seed, uint64_t offset, uint32_t b, uint32_t j) {
  const uint4 r = philox4x32_10(make_uint4(b, j >> 2, (uint32_t)offset, (uint32_t)(offset >> 32)),
                                make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const uint32_t u0 = (j & 2) ? r.z : r.x, u1 = (j & 2) ? r.w : r.y;
  float c, s;
  box_muller(u0, u1, c, s);
  return (j & 1) ? s : c;
}

// the 4 normals j = j0 .. j0+3 (j0 % 4 == 0) of philox_normal from ONE Philox block — the same
// counter, words and Box-Muller pairs, so bit-identical to four philox_normal calls
__device__ __forceinline__ f32x4 philox_normal4(uint64_t seed, uint64_t offset, uint32_t b, uint32_t j0) {
  const uint4 r = philox4x32_10(make_uint4(b, j0 >> 2, (uint32_t)offset, (uint32_t)(offset >> 32)),
                                make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  f32x4 out;
  const uint32_t us[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float c, s;
    box_muller(us[2 * h], us[2 * h + 1], c, s);
    out[2 * h] = c;
    out[2 * h + 1] = s;
  }
  return out;
}

// Wave index as a SCALAR: threadIdx-derived values are divergent to the compiler, so a plain
// `threadIdx.x >> 6` puts every quantity derived from it (column group, trip counts, weight
// addresses) in VGPRs with exec-masked loops; readfirstlane makes them SGPR/SALU work.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// ------------------------------------------------------------------ wave reduction
// Sum over the wave in a fixed order (deterministic): DPP within each 16-lane row (quad xor 1,
// quad xor 2, half-row mirror, row mirror: every lane then holds its row's sum), then the four
// row sums read out as scalars — 4 DPP adds and 4 readlanes instead of 6 ds_bpermute round trips.
// The result is wave-uniform.
#define CVAE_DPP_ADD(v, ctrl) \
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, 0xF, 0xF, false))
__device__ __forceinline__ float wave_sum(float v) {
  CVAE_DPP_ADD(v, 0xB1);   // quad_perm [1,0,3,2]
  CVAE_DPP_ADD(v, 0x4E);   // quad_perm [2,3,0,1]
  CVAE_DPP_ADD(v, 0x141);  // row_half_mirror
  CVAE_DPP_ADD(v, 0x140);  // row_mirror
  auto rd = [](float x, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
  };
  return (rd(v, 0) + rd(v, 16)) + (rd(v, 32) + rd(v, 48));
}
#undef CVAE_DPP_ADD

// k of a block whose max has biased exponent e: 2^k puts the max in [128, 256); 0 for an all-zero block
__device__ __forceinline__ int mx_k(int e) { return e > 0 ? min(134 - e, 126) : 0; }
// The lane's four quarters of 8 values (the wide chain's dX: gradient chunks in frag_k order; the MX
// dW: 8 batch rows of one feature) → e4m3 bytes of 2^k·g, k of the quarter's block; returns the two block exponents of the lane's pair (halves 0, 1 as two u16).  The
// maxima are taken on the bf16 bit patterns (|x| = bits & 0x7fff orders like the values; the bf16
// exponent field is fp32's), the pair's in one permlane16 swap (lanes L, L ^ 16), no LDS round trip.
__device__ __forceinline__ unsigned mx_block(const bf16x8 (&c)[4], l2& x0, l2& x1) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  unsigned eb[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    u16x2 m = {0, 0};
#pragma unroll
    for (int i = 2 * hh; i < 2 * hh + 2; ++i) {
      const u32x4 w = __builtin_bit_cast(u32x4, c[i]);
#pragma unroll
      for (int t = 0; t < 4; ++t) m = __builtin_elementwise_max(m, __builtin_bit_cast(u16x2, w[t] & 0x7fff7fffu));
    }
    eb[hh] = (unsigned)(m[0] > m[1] ? m[0] : m[1]) >> 7;  // biased exponent of the half's max (0: zero)
  }
  const unsigned p0 = eb[0] | eb[1] << 16;
  const auto sw = __builtin_amdgcn_permlane16_swap(p0, p0, false, false);
  const u16x2 p = __builtin_elementwise_max(__builtin_bit_cast(u16x2, (unsigned)sw[0]),
                                            __builtin_bit_cast(u16x2, (unsigned)sw[1]));
  // v_cvt_scalef32_pk_fp8_bf16 divides by its scale and rounds once (scripts/ubench/scalecvt.hip:
  // bit-equal to RNE(x·2^k) over every bf16 input, e4m3 denormals included), so 2 bf16 → 2 e4m3
  // per instruction with scale 2^−k; the block max lands in [128, 256): no saturation is needed
  typedef short i16x2 __attribute__((ext_vector_type(2)));
  long f[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float sinv = __builtin_bit_cast(float, (unsigned)(127 - mx_k(p[i >> 1])) << 23);  // 2^-k
    // the operands as shufflevector pairs: a bit_cast of one dword of the vector made the compiler
    // convert the first dword four times (hipcc of ROCm 7.2)
    const bf16x8 x = c[i];
    i16x2 lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(i16x2{0, 0}, __builtin_shufflevector(x, x, 0, 1), sinv, false);
    lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(lo, __builtin_shufflevector(x, x, 2, 3), sinv, true);
    i16x2 hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(i16x2{0, 0}, __builtin_shufflevector(x, x, 4, 5), sinv, false);
    hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(hi, __builtin_shufflevector(x, x, 6, 7), sinv, true);
    f[i] = (long)__builtin_bit_cast(unsigned, lo) | ((long)__builtin_bit_cast(unsigned, hi) << 32);
  }
  x0 = l2{f[0], f[1]};
  x1 = l2{f[2], f[3]};
  return __builtin_bit_cast(unsigned, p);
}
// one block-scaled MFMA over two 16-B e4m3 halves per operand; sa, sb: this lane's E8M0 scales
__device__ __forceinline__ f32x4 mx_mfma(l2 a0, l2 a1, l2 b0, l2 b1, f32x4 acc, int sa, int sb) {
  typedef long l4 __attribute__((ext_vector_type(4)));
  const i32x8 a = __builtin_bit_cast(i32x8, l4{a0[0], a0[1], a1[0], a1[1]});
  const i32x8 b = __builtin_bit_cast(i32x8, l4{b0[0], b0[1], b1[0], b1[1]});
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa, 0, sb);
}
