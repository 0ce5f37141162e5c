// cvae_f32chain.h — the fp32 training row chain of the reference's own configuration
// (Training_VAE.py:274-282: seq_len 10, dim 3, latent 8, hidden 128, 4+4 layers, fp32 on the sce1
// data; BASELINE configs[0]).
//
// Same work and the same arena outputs as rowchain_kernel<float, 16, RC_TRAIN> (relative transform
// :345-348, forward :169-226, reparameterisation, conditional_vae_loss :229-268 and dL/drecon, every
// dX; the tile-major xT/gT arena rows the dW kernel reduces), for one 16-row batch tile per workgroup,
// as straight-line code.  What is fp32-specific:
//  * SWAPPED fp32 MFMA: acc = W·Xᵀ with v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf chain,
//    MI355X_MICROARCH.md).  The A operand is the weight fragment exactly as the fp32 operand copies
//    store it (cvae_device.h frag_off<float>: lane (r, q) holds W[16t + r][16c + 4q + e]); the B
//    operand lane (b, q) holds X[row b][16c + 4q + e].  The accumulator of n-tile t then holds, in
//    lane (b, q), outputs 16t + 4q + i of row b — which IS the B fragment of K chunk t of the next
//    layer.  LDS images are therefore fragment images (chunk c = 1 KB, lane slot 16 B): an epilogue
//    stores one ds_write_b128, a GEMM reads one ds_read_b128 per chunk, no transposes;
//  * the ReLU mask of (row b, features 16t + 4q .. +3) is a nibble of the lane that produced it, and
//    the backward step that masks that gradient runs the same n-tile on the same lane;
//  * ONE WEIGHT STREAM per wave (as cvae_widechain.h): the 125 fragments (1 KB each) a wave multiplies
//    over the 20 GEMM steps flow through a P-deep register ring, refilled P items ahead across step
//    barriers; every offset is compile-time from the arena base (Layout below, checked against the
//    handle by plan_f32c);
//  * the two small-N steps (fc: 16 outputs, the last decoder layer: 32) split K over the 8 waves and
//    reduce the partial tiles through LDS in a fixed order (deterministic); wave 0 forms z from the fc
//    partials while every wave multiplies the h_c part of the decoder input (chunks 1..8), and z's
//    chunk 0 follows behind one more barrier;
//  * arena stores: a quad transpose (4 DPP) turns a lane's 4 features of one row into 4 rows of one
//    feature, one 16-B write-through store per lane (a wave stores 1 KB contiguous).
// MFMA work per workgroup: 500 v_mfma_f32_16x16x4_f32 per wave (fp32 MFMA is 1/16 of the bf16 rate),
// ≈13 us at 2 waves per SIMD: the 16-row form is MFMA-issue bound, the weight stream (1 MB per
// workgroup) fits under it.
// The 4-row form (RR = 4, the default up to 1,024 rows: cvae_capi.hip f32c_rows) runs the same
// stream, images and arena with v_mfma_f32_4x4x1_16b_f32 (8 instead of 32 cycles; 4 rows, K split
// over the four 16-lane groups, summed by kred).  It leaves the per-CU weight stream as the bound
// (DESIGN §4.8 "Round 6, last").
#pragma once
#include <type_traits>
#include "cvae_widechain.h"

namespace f32c {

using fchain::H;
using fchain::lbar;
using fchain::NT;
using fchain::NW;
using fchain::quad_t;
using fchain::R;
using fchain::Z;
using wchain::ArenaDst;
using wchain::arena_dst;
using wchain::sfor;

enum { LC0 = 0, LC1, LE0, LE1, LE2, LE3, LFC, LD0, LD1, LD2, LD3, NL };
// ReLU masks (nibble index): C0 C1 E0..E3 D0..D2
enum { MC0 = 0, MC1, ME0, ME1, ME2, ME3, MD0, MD1, MD2 };

// the reference architecture (latent 8, hidden 128, 4 + 4 layers) at seq_len S, dim D with
// 16 < S·D <= 32: the encoder input and the decoder output are one 32-wide padded block (two 16-wide
// fp32 K chunks / n-tiles)
template <int S_, int D_>
struct Arch {
  static constexpr int S = S_, D = D_, I = S_ * D_, Ip = 32;
  static_assert(I > 16 && I <= 32 && D >= 3, "S*D in (16, 32]; channels 0..2 = t, x, y");
  static constexpr int Kp(int l) { return l == LC0 ? 32 : l == LE0 ? Ip : l == LFC ? 2 * H : l == LD0 ? 160 : H; }
  static constexpr int Np(int l) { return l == LFC ? 32 : l == LD3 ? Ip : H; }
  // the arena as alloc_arena (cvae_capi.hip) lays it out for fp32 operands: byte offsets from its base
  static constexpr int64_t r256(int64_t b) { return (b + 255) / 256 * 256; }
  static constexpr int64_t wf(int l) {
    int64_t o = 0;
    for (int k = 0; k < l; ++k) o += 2 * r256(4LL * Np(k) * Kp(k));
    return o;
  }
  static constexpr int64_t wb(int l) { return wf(l) + r256(4LL * Np(l) * Kp(l)); }
  static constexpr int bias_off(int l) {
    int o = 0;
    for (int k = 0; k < l; ++k) o += Np(k);
    return o;
  }
  static constexpr int nbias = bias_off(NL);
  static constexpr int64_t bias_base = wf(NL);
  static constexpr int64_t act0 = bias_base + r256(4LL * nbias);
  static constexpr int64_t xrows(int l) {  // xT(l) = act0 + 4·Bp·xrows(l) (Bp % 32 == 0)
    int64_t o = 0;
    for (int k = 0; k < l; ++k) o += Kp(k) + Np(k);
    return o;
  }
  static constexpr int64_t grows(int l) { return xrows(l) + Kp(l); }
  // LDS (bytes): fragment images, 1 KB per 16 features
  static constexpr int L_XIN = 0,                 // x_rel (2 chunks), then dL/drecon in place
      L_CIN = L_XIN + 2048,                       // condition input [start x, start y, 0..] (1 chunk)
      L_CB = L_CIN + 1024,                        // C0 output; in the backward dh_c (C1ᵀ's input)
      L_A0 = L_CB + 8192, L_A1 = L_A0 + 8192,     // hidden ping-pong
      L_HCAT = L_A1 + 8192,                       // [h_traj ‖ h_c] (16 chunks)
      L_DCAT = L_HCAT + 16384,                    // [z ‖ h_c ‖ 0] (9 chunks; z only in registers)
      L_GFC = L_DCAT + 9 * 1024,                  // [dmu ‖ dlogvar]
      L_DHC2 = L_GFC + 1024,                      // the decoder's share of dh_c, h_c-aligned (8 chunks)
      L_PART = L_DHC2 + 8192,                     // K-split partial tiles [wave][1 KB]
      L_RCH0 = L_PART + 8192,                     // fp32 [s][row]: recon time channel
      L_GD0 = L_RCH0 + S * R * 4,                 // fp32 [s][row]: its dL/drecon before the fix-up
      L_BIAS = L_GD0 + S * R * 4, L_LP = L_BIAS + nbias * 4, L_STAMPS = L_LP + NW * 8 * 4,
      L_TOTAL = L_STAMPS + (CVAE_DIAG_STAMPS ? 64 * 8 : 0);
  static_assert(L_TOTAL <= 160 * 1024, "LDS");
};

// ---- the weight stream: the GEMM steps in consumption order and their 1-KB items per wave
enum { sC0, sE0, sC1, sE1, sE2, sE3, sFC, sD0, sD1, sD2, sD3, sD3b, sD2b, sD1b, sD0b, sFCb, sE3b, sE2b, sE1b, sC1b, NS };
constexpr int layer_of(int s) {
  return s == sC0 ? LC0 : s == sE0 ? LE0 : s == sC1 || s == sC1b ? LC1 : s == sE1 || s == sE1b ? LE1
       : s == sE2 || s == sE2b ? LE2 : s == sE3 || s == sE3b ? LE3 : s == sFC || s == sFCb ? LFC
       : s == sD0 || s == sD0b ? LD0 : s == sD1 || s == sD1b ? LD1 : s == sD2 || s == sD2b ? LD2 : LD3;
}
constexpr bool bwd_of(int s) { return s >= sD3b; }
// C0: one chunk (K = 2); E0, fc and the last decoder layer (K split), D3ᵀ (K = 32), fcᵀ (K = 16, two
// n-tiles): 2; decoder L0 forward (K = 136 → 9 chunks) and backward (tile + the K-split tile 8): 9
constexpr int nitems(int s) {
  return s == sC0 ? 1 : (s == sE0 || s == sFC || s == sD3 || s == sD3b || s == sFCb) ? 2 : (s == sD0 || s == sD0b) ? 9 : 8;
}
constexpr int start(int s) {
  int g = 0;
  for (int k = 0; k < s; ++k) g += nitems(k);
  return g;
}
constexpr int TOTAL = start(NS);
constexpr int step_of(int g) {
  int s = 0;
  while (s + 1 < NS && start(s + 1) <= g) ++s;
  return s;
}
static_assert(TOTAL == 125, "items per wave");

// byte offset (from the arena base) of item j of step s for wave w: fragment (n-tile t, chunk c) of
// the operand at (t·KCH + c) KB
template <class A, int s, int j>
__device__ __forceinline__ int item_off(int w) {
  constexpr int l = layer_of(s);
  constexpr int64_t base = bwd_of(s) ? A::wb(l) : A::wf(l);
  constexpr int kch = (bwd_of(s) ? A::Np(l) : A::Kp(l)) / 16;
  int frag;
  if constexpr (s == sFC) frag = 2 * w + j;                                // tile 0, chunks 2w, 2w+1
  else if constexpr (s == sD3) frag = (w >> 2) * kch + 2 * (w & 3) + j;   // tile w/4, chunks 2(w%4), +1
  else if constexpr (s == sD0) frag = w * kch + (j < 8 ? j + 1 : 0);     // chunks 1..8, then 0 (z)
  else if constexpr (s == sD0b) frag = j < 8 ? w * kch + j : 8 * kch + w; // tile w; tile 8 chunk w
  else if constexpr (s == sFCb) frag = (j == 0 ? w : 8 + w) * kch;        // tiles w, 8+w, chunk 0
  else frag = w * kch + j;                                                // tile w, chunk j
  return (int)base + frag * 1024;
}

template <int P>
struct Ring {
  f32x4 r[P];
};
// stream item G of this wave → ring slot G % P (no-op past the end): a buffer load, lane·16 the
// voffset and the item's offset a scalar soffset
template <class A, int P, int G>
__device__ __forceinline__ void ring_load(Ring<P>& ring, const char* AR, int wave, int lane) {
  if constexpr (G < TOTAL) {
    constexpr int s = step_of(G), j = G - start(s);
    int w = wave;
    asm volatile("" : "+s"(w));  // per item: hoisted, every item's offset would be a live SGPR
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)AR, (short)0, 0x7fffffff, 0x00020000);
    ring.r[G % P] = CVAE_DIAG_NOWLOAD ? f32x4{}
                                      : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                      rs, lane * 16, item_off<A, s, j>(w), 0));
  }
}

// acc += W·Xᵀ over one 16-wide K chunk (element e of both fragments).  RR = 16: four 16x16x4 fp32
// MFMAs.  RR = 4: four v_mfma_f32_4x4x1_16b_f32 — the weight fragment's lane (r, kg) is A row r % 4 of
// block 4kg + r / 4, so block 4kg + m multiplies features 16t + 4m .. +3 by the X value of k
// 16c + 4kg + e of rows 0..3 (B lanes (kg, m, j)); the result holds only k-group kg's share of the
// chunk (kred sums the four groups)
template <int RR>
__device__ __forceinline__ f32x4 mm4(f32x4 w, f32x4 x, f32x4 acc) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
    acc = RR == 4 ? __builtin_amdgcn_mfma_f32_4x4x1f32(w[e], x[e], acc, 0, 0, 0)
                  : __builtin_amdgcn_mfma_f32_16x16x4f32(w[e], x[e], acc, 0, 0, 0);
  return acc;
}
// RR = 4: the four k-groups' partial sums (lanes 16 and 32 apart), every lane the same total
// ((P0 + P1) + (P2 + P3) in any lane: fp32 addition commutes).  gfx950's row swaps (VALU, no LDS
// round trip): v_permlane16_swap of v with itself leaves one copy holding rows (0, 0, 2, 2) and the
// other (1, 1, 3, 3), so their sum is the pair sum of rows 16 apart in every lane; v_permlane32_swap
// does the same for the halves.  CVAE_F32_KRED_SWAP=0: the ds_bpermute butterfly (bit-equal).
#ifndef CVAE_F32_KRED_SWAP
#define CVAE_F32_KRED_SWAP 1
#endif
__device__ __forceinline__ f32x4 kred(f32x4 v) {
#if CVAE_F32_KRED_SWAP
  auto u = [](float f) { return __builtin_bit_cast(unsigned, f); };
  auto f = [](unsigned x) { return __builtin_bit_cast(float, x); };
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(u(v[i]), u(v[i]), false, false);
    v[i] = f(r[0]) + f(r[1]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto r = __builtin_amdgcn_permlane32_swap(u(v[i]), u(v[i]), false, false);
    v[i] = f(r[0]) + f(r[1]);
  }
#else
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] += __shfl_xor(v[i], 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] += __shfl_xor(v[i], 32);
#endif
  return v;
}
// the B operand (X fragment) of chunk c: RR = 16 lane (b, q) reads slot (q, b), its own lane's;
// RR = 4 lane (kg, m, j) reads slot (kg, j)
template <int RR>
__device__ __forceinline__ f32x4 ldsB(const char* img, int c) {
  const int lane = threadIdx.x & 63;
  return *(const f32x4*)(img + c * 1024 + (RR == 4 ? (lane & 48) + (lane & 3) : lane) * 16);
}
// slot (quad q, row b) of chunk c
__device__ __forceinline__ f32x4 lds_slot(const char* img, int c, int q, int b) {
  return *(const f32x4*)(img + c * 1024 + (q * 16 + b) * 16);
}
__device__ __forceinline__ void sts_slot(char* img, int c, int q, int b, f32x4 v) {
  *(f32x4*)(img + c * 1024 + (q * 16 + b) * 16) = v;
}

// Items [J0, J1) of step s: item j multiplies the ring slot of its stream index by the X fragment of
// chunk xc(j) (all read first), two accumulators alternating (the 16x16x4 MFMA's dependent latency is
// 40 cycles against a 32-cycle issue); each consumed slot is refilled P items ahead.  xr(j, x) may
// replace a fragment (the decoder input's z lanes).
struct NoX {
  __device__ f32x4 operator()(int, f32x4 x) const { return x; }
};
template <class A, int RR, int P, int s, int J0, int J1, class XC, class XR = NoX>
__device__ __forceinline__ f32x4 gemm(Ring<P>& ring, const char* img, XC xc, const char* AR, int wave, int lane,
                                      XR xr = XR{}) {
  constexpr int G0 = start(s), N = J1 - J0;
  f32x4 x[N];
  sfor<J0, J1>([&](auto jj) {
    constexpr int j = decltype(jj)::value;
    x[j - J0] = xr(j, ldsB<RR>(img, xc(j)));
  });
  if constexpr (RR == 4) {  // four independent accumulators (element e), k-groups summed at the end
    f32x4 a[4] = {};
    sfor<J0, J1>([&](auto jj) {
      constexpr int j = decltype(jj)::value, g = G0 + j;
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = __builtin_amdgcn_mfma_f32_4x4x1f32(ring.r[g % P][e], x[j - J0][e], a[e], 0, 0, 0);
      asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
      ring_load<A, P, g + P>(ring, AR, wave, lane);
    });
    return kred((a[0] + a[1]) + (a[2] + a[3]));
  }
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  sfor<J0, J1>([&](auto jj) {
    constexpr int j = decltype(jj)::value, g = G0 + j;
    if constexpr ((j - J0) & 1) {
      a1 = mm4<16>(ring.r[g % P], x[j - J0], a1);
      asm volatile("" : "+v"(a1));  // MFMA(g) before refill(g + P): the slot is not held twice
    } else {
      a0 = mm4<16>(ring.r[g % P], x[j - J0], a0);
      asm volatile("" : "+v"(a0));
    }
    ring_load<A, P, g + P>(ring, AR, wave, lane);
  });
  return N > 1 ? a0 + a1 : a0;
}

template <class A, int P, int RR>
__device__ __forceinline__ void f32_body(char* const AR, const int Bp, const RowArgs& a, char* smem, int blk) {
  static_assert(RR == 16 || RR == 4, "row tiles of 16 or 4");
  constexpr int S = A::S, D = A::D, I = A::I;
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  // a lane's output slot: row b, features 16t + 4q .. +3 of its wave's n-tile t.  RR = 16: lane
  // (b, q).  RR = 4: lane (kg, q, b) — after kred the four k-groups hold the same values and only
  // k-group 0 (`own`) writes them
  const int b = RR == 4 ? lane & 3 : lane & 15, q = RR == 4 ? (lane >> 2) & 3 : lane >> 4;
  const bool own = RR == 4 ? lane < 16 : true;
  const int b0 = blk * RR, nrows = max(0, min(RR, a.batch - b0));
  char* const XIN = smem + A::L_XIN;
  char* const CIN = smem + A::L_CIN;
  char* const CB = smem + A::L_CB;
  char* const A0 = smem + A::L_A0;
  char* const A1 = smem + A::L_A1;
  char* const HCAT = smem + A::L_HCAT;
  char* const DCAT = smem + A::L_DCAT;
  char* const GFC = smem + A::L_GFC;
  char* const DHC2 = smem + A::L_DHC2;
  char* const PART = smem + A::L_PART;
  float* const RCH0 = (float*)(smem + A::L_RCH0);
  float* const GD0 = (float*)(smem + A::L_GD0);
  float* const BIAS = (float*)(smem + A::L_BIAS);
  float* const LP = (float*)(smem + A::L_LP);
  unsigned long long* const STAMPS = (unsigned long long*)(smem + A::L_STAMPS);
  int stamp_i = 0;
  auto bar = [&]() {
    lbar();
    if (CVAE_DIAG_STAMPS && threadIdx.x == 0 && stamp_i < 64) STAMPS[stamp_i] = __builtin_amdgcn_s_memrealtime();
    ++stamp_i;
  };
  if (CVAE_DIAG_STAMPS && threadIdx.x == 0) STAMPS[stamp_i++] = __builtin_amdgcn_s_memrealtime();
  const ArenaDst dst = arena_dst(AR);
  // arena matrices: byte offsets recomputed from Bp (one SGPR) at each use
  auto XT = [&](int l) -> int {
    int bp = Bp;
    asm volatile("" : "+s"(bp));
    return (int)(A::act0 + 4 * (int64_t)bp * A::xrows(l));
  };
  auto GT = [&](int l) -> int {
    int bp = Bp;
    asm volatile("" : "+s"(bp));
    return (int)(A::act0 + 4 * (int64_t)bp * A::grows(l));
  };
  // this lane's 4 values (row b, features F .. F+3) of an arena matrix (byte offset mat, Kf feature
  // rows): the quad transpose gives lane b = 4j + m feature F + m of rows 4j .. 4j+3, one 16-B
  // write-through store (a wave instruction covers 16 features x 16 rows: 1 KB contiguous).  Every
  // lane of the wave must run it (DPP); `on` predicates the store only.
  // (RR = 4: the quad is rows 0..3 of one feature quad; the workgroup's 4 rows are rows
  // 4(blk % 4) .. +3 of 16-row arena tile blk / 4)
  auto ast = [&](int mat, int Kf, int F, f32x4 v, bool on = true) {
    const f32x4 t = quad_t(v);
    const int off = RR == 4 ? (((blk >> 2) * Kf + F + b) * 16 + (blk & 3) * 4) * 4
                            : ((blk * Kf + F + (b & 3)) * 16 + (b & ~3)) * 4;
    if (on && own && !CVAE_DIAG_NOSTORE)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, t), dst.rs, mat + off, 0, 16);
  };
  // a fragment image's features [0, NF) to an arena matrix (tasks t = 0 .. 4·NF-1: feature t/4, rows
  // 4(t%4) .. +3 — four LDS dwords, one 16-B store)
  auto img_arena = [&](const char* img, int NF, int mat, int Kf, int goff, int t) {
    constexpr int TPF = RR / 4;  // 4-row tasks per feature
    if (t < 0 || t >= TPF * NF || CVAE_DIAG_NOSTORE) return;
    const int f = t / TPF, j = t % TPF;
    const float* p = (const float*)(img + ((f >> 4) * 64 + ((f & 15) >> 2) * 16 + 4 * j) * 16) + (f & 3);
    const f32x4 v = {p[0], p[4], p[8], p[12]};
    const int off = RR == 4 ? (((blk >> 2) * Kf + goff + f) * 16 + (blk & 3) * 4) * 4 : ((blk * Kf + goff + f) * 16 + 4 * j) * 4;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), dst.rs, mat + off, 0, 16);
  };
  // this lane's output slot (row b, features 16c + 4q .. +3) of image chunk c
  auto sto = [&](char* img, int c, f32x4 v) {
    if (own) sts_slot(img, c, q, b, v);
  };
  auto bias4 = [&](int l, int f) { return *(const f32x4*)(BIAS + A::bias_off(l) + f); };

  // ReLU masks: nibble M (this lane: row b, features 16·wave + 4q .. +3) at bits 4M
  uint64_t mk = 0;
  auto relu = [&](f32x4 acc, f32x4 bb, auto m) {
    constexpr int M = decltype(m)::value;
    f32x4 y;
    uint64_t nib = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y[i] = fmaxf(acc[i] + bb[i], 0.f);
      nib |= (uint64_t)(y[i] > 0.f ? 1u : 0u) << i;
    }
    mk |= nib << (4 * M);
    asm volatile("" : "+v"(mk));  // materialised now: the activations are not kept for the backward
    return y;
  };
  auto masked = [&](f32x4 g, auto m) {
    constexpr int M = decltype(m)::value;
    const uint32_t nib = (uint32_t)(mk >> (4 * M));
    f32x4 y;
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = (nib >> i) & 1u ? g[i] : 0.f;
    return y;
  };
  using std::integral_constant;
  auto cid = [](int j) { return j; };
  const int n4 = 16 * wave + 4 * q;  // this lane's first feature in the 128-wide layers (n-tile = wave)

  // the Philox offset of this launch (scalar load first)
  const uint64_t rng_off = a.ctr ? *(const __attribute__((address_space(4))) uint64_t*)a.ctr : a.offset;
  Ring<P> ring;
  float s_recon = 0.f, s_kl = 0.f, s_start = 0.f, s_t0 = 0.f, s_relu = 0.f;
  f32x4 ep;  // eps of (row b, latents 4(q & 1) .. +3) — lanes q < 2 use theirs (every wave forms z)

  // ================================================================ prologue
  {
    const int last = max(a.batch - 1, 0);
    // x tile: thread t < 256 loads the feature pair (2p, 2p+1) of row r = t / 16 (8-B loads: an fp32 row
    // of S·D = 30 floats is 8-B aligned) and the row's start point x[:, 0, 1:3] (:345)
    const int xr = tid >> 4, xp = tid & 15;
    u32x2 xv = {0u, 0u};
    float sx = 0.f, sy = 0.f;
    if (tid < 16 * RR) {  // wave-uniform
      int64_t g = min(b0 + xr, last);
      if (a.idx) g = gld<int64_t>(a.idx + g);
      const float* const row = (const float*)a.x + g * I;
      if (2 * xp < I) xv = gld<u32x2>(row + 2 * xp);
      sx = gld<float>(row + 1);
      sy = gld<float>(row + 2);
    }
    // host eps (loaded unconditionally, rows clamped into the batch: a load under a branch drains the
    // weight stream)
    const int erow = a.eps ? min(b0 + b, last) : 0;
    const f32x4 eh = gld<f32x4>((a.eps ? a.eps : (const float*)(AR + A::bias_base)) + (a.eps ? (size_t)erow * Z + 4 * (q & 1) : 0));
    constexpr int NB4 = A::nbias / 4;
    f32x4 bv0 = {}, bv1 = {};
    const int kb = tid - 256;
    if (kb >= 0 && kb < NB4) bv0 = gld<f32x4>((const float*)(AR + A::bias_base) + 4 * kb);
    if (kb >= 0 && kb + 256 < NB4) bv1 = gld<f32x4>((const float*)(AR + A::bias_base) + 4 * (kb + 256));
    sfor<0, P>([&](auto g) { ring_load<A, P, decltype(g)::value>(ring, AR, wave, lane); });
    // eps while the x tile is in flight (wave 0, which forms z): Philox keyed by the GLOBAL row
    // (eps_row0 = a rank's first row)
    ep = f32x4{0.f, 0.f, 0.f, 0.f};
    if (wave == 0) {
      const f32x4 d = philox_normal4(a.seed, rng_off, (uint32_t)(a.eps_row0 + b0 + b), (uint32_t)(4 * (q & 1)));
      ep = a.eps ? eh : d;
      if (b >= nrows) ep = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // device counters: this launch begins optimizer step ctr[1] + 1 and precomputes its Adam scalars
    // (one wave of block 0, wave-uniformly; one lane stores)
    if (a.ctr && blk == 0 && wave == NW - 1) {
      const uint64_t t = *(const __attribute__((address_space(4))) uint64_t*)(a.ctr + 1) + 1;
      float c0 = 0.f, c1 = 0.f;
      if (a.adam_pre) adam_scalars(a.lr, a.beta1, a.beta2, (double)t, c0, c1);
      if (lane == 0) {
        __hip_atomic_store(a.ctr + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.adam_pre)
          __hip_atomic_store(a.ctr + 2, __builtin_bit_cast(uint64_t, adam_f32x2{c0, c1}), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (kb >= 0 && kb < NB4) ((f32x4*)BIAS)[kb] = bv0;
    if (kb >= 0 && kb + 256 < NB4) ((f32x4*)BIAS)[kb + 256] = bv1;
    // the decoder input's K padding (features 136..143: chunk 8, quads 2, 3) is read by D0
    if (tid >= 256 && tid < 256 + 32) sts_slot(DCAT, 8, 2 + ((tid - 256) >> 4), (tid - 256) & 15, f32x4{0.f, 0.f, 0.f, 0.f});
    if (tid < 16 * RR) {
      // the relative transform in fp32 (:345-348): channels 1, 2 minus the start point; rows past the
      // batch are zero
      const bool live = xr < nrows;
      const int f0 = 2 * xp;
      auto rebase = [&](uint32_t u, int f) {
        const float x = __builtin_bit_cast(float, u);
        const int d = f % D;
        return (!live || f >= I) ? 0.f : d == 1 ? x - sx : d == 2 ? x - sy : x;
      };
      const float v0 = rebase(xv.x, f0), v1 = rebase(xv.y, f0 + 1);
      // features f0, f0 + 1 of row xr: chunk f0 / 16, quad (f0 % 16) / 4, elements f0 % 4, +1
      *(u32x2*)(XIN + ((f0 >> 4) * 64 + ((f0 & 15) >> 2) * 16 + xr) * 16 + (f0 & 3) * 4) =
          u32x2{__builtin_bit_cast(uint32_t, v0), __builtin_bit_cast(uint32_t, v1)};
      if (xp < 4) {  // the condition input (x, y) of the row (c_start, :345): CIN features 0, 1
        const f32x4 c = xp == 0 && live ? f32x4{sx, sy, 0.f, 0.f} : f32x4{0.f, 0.f, 0.f, 0.f};
        sts_slot(CIN, 0, xp, xr, c);
      }
    }
  }
  bar();

  const float Bf = (float)a.batch;
  const float inv_BSD = 1.f / (Bf * (float)(S * D)), inv_2B = 1.f / (2.f * Bf), inv_B = 1.f / Bf;
  const float inv_BS1 = S > 1 ? 1.f / (Bf * (float)(S - 1)) : 0.f, inv_BZ = 1.f / (Bf * (float)Z);
  const bool use_start = a.w_start > 0.f, use_time = a.w_time > 0.f;  // Training_VAE.py:247, :256

  // ================================================================ forward
  {  // C0 ‖ E0 (:132-137, :141-151)
    f32x4 acc = gemm<A, RR, P, sC0, 0, 1>(ring, CIN, cid, AR, wave, lane);
    f32x4 y = relu(acc, bias4(LC0, n4), integral_constant<int, MC0>{});
    sto(CB, wave, y);
    ast(XT(LC1), H, n4, y);
    acc = gemm<A, RR, P, sE0, 0, 2>(ring, XIN, cid, AR, wave, lane);
    y = relu(acc, bias4(LE0, n4), integral_constant<int, ME0>{});
    sto(A0, wave, y);
    ast(XT(LE1), H, n4, y);
    img_arena(XIN, 32, XT(LE0), A::Kp(LE0), 0, tid);        // x_rel → xT(E0)
    img_arena(CIN, 16, XT(LC0), A::Kp(LC0), 0, tid - 128);  // (x, y, 0..) → xT(C0)
  }
  bar();
  {  // C1 ‖ E1: h_c into both concatenations (fc input at H + n, decoder input at Z + n)
    f32x4 acc = gemm<A, RR, P, sC1, 0, 8>(ring, CB, cid, AR, wave, lane);
    const f32x4 hc = relu(acc, bias4(LC1, n4), integral_constant<int, MC1>{});
    sto(HCAT, 8 + wave, hc);
    if (own) sts_slot(DCAT, wave + (q >> 1), (q + 2) & 3, b, hc);  // decoder-input feature Z + n4
    ast(XT(LFC), A::Kp(LFC), H + n4, hc);
    ast(XT(LD0), A::Kp(LD0), Z + n4, hc);
    acc = gemm<A, RR, P, sE1, 0, 8>(ring, A0, cid, AR, wave, lane);
    const f32x4 y = relu(acc, bias4(LE1, n4), integral_constant<int, ME1>{});
    sto(A1, wave, y);
    ast(XT(LE2), H, n4, y);
  }
  bar();
  {  // E2
    const f32x4 acc = gemm<A, RR, P, sE2, 0, 8>(ring, A1, cid, AR, wave, lane);
    const f32x4 y = relu(acc, bias4(LE2, n4), integral_constant<int, ME2>{});
    sto(A0, wave, y);
    ast(XT(LE3), H, n4, y);
  }
  bar();
  {  // E3 → h_traj
    const f32x4 acc = gemm<A, RR, P, sE3, 0, 8>(ring, A0, cid, AR, wave, lane);
    const f32x4 y = relu(acc, bias4(LE3, n4), integral_constant<int, ME3>{});
    sto(HCAT, wave, y);
    ast(XT(LFC), A::Kp(LFC), n4, y);
  }
  bar();
  {  // fc_mu ‖ fc_logvar (:195-196): one n-tile, K chunks 2w, 2w+1 per wave → partial tiles
    const f32x4 acc = gemm<A, RR, P, sFC, 0, 2>(ring, HCAT, [wave](int j) { return 2 * wave + j; }, AR, wave, lane);
    sto(PART, wave, acc);
  }
  bar();
  // D0 over [z ‖ h_c]: every wave multiplies the h_c chunks 1..8 while wave 0 forms mu, logvar (lanes
  // q < 2: latents 4q .. 4q+3 of row b) from the fc partials in a fixed order, reparameterizes
  // (:199-206) and writes z into chunk 0; chunk 0 after one more barrier
  f32x4 mu = {}, lv = {}, zz = {};
  f32x4 acc0;
  {
    if (wave == 0) {
      const int qq = q & 1;
      f32x4 sm = lds_slot(PART, 0, qq, b), sl = lds_slot(PART, 0, qq + 2, b);
#pragma unroll
      for (int v = 1; v < NW; ++v) {
        sm += lds_slot(PART, v, qq, b);
        sl += lds_slot(PART, v, qq + 2, b);
      }
      mu = sm + bias4(LFC, 4 * qq);
      lv = sl + bias4(LFC, Z + 4 * qq);
#pragma unroll
      for (int i = 0; i < 4; ++i) zz[i] = mu[i] + ep[i] * expf(0.5f * lv[i]);
      if (q < 2 && own) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (b < nrows) s_kl += 1.f + lv[i] - mu[i] * mu[i] - expf(lv[i]);  // KL (:243)
        sts_slot(DCAT, 0, q, b, zz);
      }
    }
    acc0 = gemm<A, RR, P, sD0, 0, 8>(ring, DCAT, [](int j) { return j + 1; }, AR, wave, lane);
    if (wave == 0) ast(XT(LD0), A::Kp(LD0), 4 * q, zz, q < 2);  // z → xT(D0) features 0..7
  }
  bar();
  {  // D0 chunk 0: [z ‖ h_c 0..7]
    const f32x4 acc = acc0 + gemm<A, RR, P, sD0, 8, 9>(ring, DCAT, [](int) { return 0; }, AR, wave, lane);
    const f32x4 y = relu(acc, bias4(LD0, n4), integral_constant<int, MD0>{});
    sto(A0, wave, y);
    ast(XT(LD1), H, n4, y);
  }
  bar();
  {  // D1
    const f32x4 acc = gemm<A, RR, P, sD1, 0, 8>(ring, A0, cid, AR, wave, lane);
    const f32x4 y = relu(acc, bias4(LD1, n4), integral_constant<int, MD1>{});
    sto(A1, wave, y);
    ast(XT(LD2), H, n4, y);
  }
  bar();
  {  // D2
    const f32x4 acc = gemm<A, RR, P, sD2, 0, 8>(ring, A1, cid, AR, wave, lane);
    const f32x4 y = relu(acc, bias4(LD2, n4), integral_constant<int, MD2>{});
    sto(A0, wave, y);
    ast(XT(LD3), H, n4, y);
  }
  bar();
  {  // D3: n-tile w / 4, K chunks 2(w % 4), +1 → partial tiles
    const f32x4 acc = gemm<A, RR, P, sD3, 0, 2>(ring, A0, [wave](int j) { return 2 * (wave & 3) + j; }, AR, wave, lane);
    sto(PART, wave, acc);
  }
  bar();
  if (wave < 2 && own) {  // recon n-tile u = wave + conditional_vae_loss (:229-268) + dL/drecon over x_rel in place
    const int u = wave;
    f32x4 r = lds_slot(PART, 4 * u, q, b);
#pragma unroll
    for (int v = 1; v < 4; ++v) r += lds_slot(PART, 4 * u + v, q, b);
    r += bias4(LD3, 16 * u + 4 * q);
    const f32x4 xr = lds_slot(XIN, u, q, b);
    const bool live = b < nrows;
    const float cr = a.w_recon * 2.f;
    f32x4 g;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = 16 * u + 4 * q + i;
      g[i] = 0.f;
      if (f < I) {
        const float d = live ? r[i] - xr[i] : 0.f;
        s_recon += d * d;
        g[i] = d * cr * inv_BSD;  // w_recon·2·diff / (B·S·D)
        const int dd = f % D;
        if (f < D && live) {  // timestep 0
          if ((dd == 1 || dd == 2) && use_start) {
            s_start += d * d;
            g[i] += a.w_start * 2.f * d * inv_2B;
          }
          if (dd == 0 && use_time) {
            s_t0 += r[i] * r[i];
            g[i] += a.w_time * 2.f * r[i] * inv_B;
          }
        }
        if (dd == 0) {
          RCH0[(f / D) * RR + b] = r[i];
          GD0[(f / D) * RR + b] = g[i];
        }
      }
    }
    sto(XIN, u, g);
  }
  bar();
  // time-monotonicity term relu(r_s − r_{s+1}) (:261-262, ReLU'(0) = 0) into the time channel of
  // dL/drecon: one task per (timestep, row)
  if (tid < S * RR) {
    const int s = tid / RR, bb = tid % RR;
    float gv = GD0[s * RR + bb];
    if (use_time) {
      const float rs = RCH0[s * RR + bb], rn = RCH0[min(s + 1, S - 1) * RR + bb], rp = RCH0[max(s - 1, 0) * RR + bb];
      const float u1 = rs - rn, u0 = rp - rs;  // 0 at the sequence ends
      if (bb < nrows && u1 > 0.f) {
        gv += a.w_time * inv_BS1;
        s_relu += u1;
      }
      if (bb < nrows && u0 > 0.f) gv -= a.w_time * inv_BS1;
    }
    const int f = s * D;
    *((float*)(XIN + ((f >> 4) * 64 + ((f & 15) >> 2) * 16 + bb) * 16) + (f & 3)) = gv;
  }
  bar();

  // ================================================================ backward
  {  // D3ᵀ: dL/d h_D2 = GL · W_D3, mask of D2
    const f32x4 acc = gemm<A, RR, P, sD3b, 0, 2>(ring, XIN, cid, AR, wave, lane);
    const f32x4 g = masked(acc, integral_constant<int, MD2>{});
    sto(A1, wave, g);
    ast(GT(LD2), H, n4, g);
    img_arena(XIN, 32, GT(LD3), A::Np(LD3), 0, tid - 256);  // dL/drecon → gT(D3)
  }
  bar();
  {  // D2ᵀ
    const f32x4 acc = gemm<A, RR, P, sD2b, 0, 8>(ring, A1, cid, AR, wave, lane);
    const f32x4 g = masked(acc, integral_constant<int, MD1>{});
    sto(A0, wave, g);
    ast(GT(LD1), H, n4, g);
  }
  bar();
  {  // D1ᵀ
    const f32x4 acc = gemm<A, RR, P, sD1b, 0, 8>(ring, A0, cid, AR, wave, lane);
    const f32x4 g = masked(acc, integral_constant<int, MD0>{});
    sto(A1, wave, g);
    ast(GT(LD0), H, n4, g);
  }
  bar();
  {  // D0ᵀ: [dz ‖ dh_c (decoder share)]; tile w over all of K, tile 8 (features 128..143) K-split
    const f32x4 acc = gemm<A, RR, P, sD0b, 0, 8>(ring, A1, cid, AR, wave, lane);
    const f32x4 p8 = gemm<A, RR, P, sD0b, 8, 9>(ring, A1, [wave](int) { return wave; }, AR, wave, lane);
    sto(PART, wave, p8);
    if (wave == 0 && q < 2) {  // dz of latents 4q .. +3 → KL / reparameterisation backward (:199-206, :243)
      f32x4 gm, gl;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool live = b < nrows;
        const float sd = expf(0.5f * lv[i]);
        gm[i] = live ? a.w_kld * mu[i] * inv_BZ + acc[i] : 0.f;
        gl[i] = live ? a.w_kld * 0.5f * (expf(lv[i]) - 1.f) * inv_BZ + acc[i] * ep[i] * 0.5f * sd : 0.f;
      }
      if (own) {
        sts_slot(GFC, 0, q, b, gm);
        sts_slot(GFC, 0, q + 2, b, gl);
      }
    } else if (own) {  // h_c features n4 - Z .. +3 → the h_c-aligned image
      const int hf = n4 - Z;
      sts_slot(DHC2, hf >> 4, (hf & 15) >> 2, b, acc);
    }
  }
  bar();
  {  // fcᵀ: dh = G_fc · W_fc → h_traj gradient (mask E3) and h_c gradient (+ decoder share, mask C1)
    const f32x4 x = ldsB<RR>(GFC, 0);
    constexpr int G0 = start(sFCb);
    f32x4 ah = mm4<RR>(ring.r[G0 % P], x, f32x4{0.f, 0.f, 0.f, 0.f});
    f32x4 ac = mm4<RR>(ring.r[(G0 + 1) % P], x, f32x4{0.f, 0.f, 0.f, 0.f});
    asm volatile("" : "+v"(ah), "+v"(ac));
    ring_load<A, P, G0 + P>(ring, AR, wave, lane);
    ring_load<A, P, G0 + 1 + P>(ring, AR, wave, lane);
    if constexpr (RR == 4) {
      ah = kred(ah);
      ac = kred(ac);
    }
    img_arena(GFC, 16, GT(LFC), A::Np(LFC), 0, tid - 256);  // [dmu ‖ dlogvar] → gT(fc)
    const f32x4 gt = masked(ah, integral_constant<int, ME3>{});
    sto(A0, wave, gt);
    ast(GT(LE3), H, n4, gt);
    f32x4 d2;  // the decoder share; h_c 120..127 (wave 7, q >= 2) is tile 8's partial sum
    if (wave == NW - 1 && q >= 2) {
      d2 = lds_slot(PART, 0, q - 2, b);
#pragma unroll
      for (int v = 1; v < NW; ++v) d2 += lds_slot(PART, v, q - 2, b);
    } else {
      d2 = lds_slot(DHC2, wave, q, b);
    }
    const f32x4 gc = masked(ac + d2, integral_constant<int, MC1>{});
    sto(CB, wave, gc);
    ast(GT(LC1), H, n4, gc);
  }
  bar();
  {  // E3ᵀ
    const f32x4 acc = gemm<A, RR, P, sE3b, 0, 8>(ring, A0, cid, AR, wave, lane);
    const f32x4 g = masked(acc, integral_constant<int, ME2>{});
    sto(A1, wave, g);
    ast(GT(LE2), H, n4, g);
  }
  bar();
  {  // E2ᵀ
    const f32x4 acc = gemm<A, RR, P, sE2b, 0, 8>(ring, A1, cid, AR, wave, lane);
    const f32x4 g = masked(acc, integral_constant<int, ME1>{});
    sto(A0, wave, g);
    ast(GT(LE1), H, n4, g);
  }
  bar();
  {  // E1ᵀ ‖ C1ᵀ: the last two gradients, gT(E0) and gT(C0), only feed the dW kernel
    f32x4 acc = gemm<A, RR, P, sE1b, 0, 8>(ring, A0, cid, AR, wave, lane);
    ast(GT(LE0), H, n4, masked(acc, integral_constant<int, ME0>{}));
    acc = gemm<A, RR, P, sC1b, 0, 8>(ring, CB, cid, AR, wave, lane);
    ast(GT(LC0), H, n4, masked(acc, integral_constant<int, MC0>{}));
  }
  // ---- loss partial sums (deterministic order)
  s_recon = wave_sum(s_recon);
  s_kl = wave_sum(s_kl);
  s_start = wave_sum(s_start);
  s_t0 = wave_sum(s_t0);
  s_relu = wave_sum(s_relu);
  if (lane == 0) {
    LP[wave * 8 + 0] = s_recon;
    LP[wave * 8 + 1] = s_kl;
    LP[wave * 8 + 2] = s_start;
    LP[wave * 8 + 3] = s_t0;
    LP[wave * 8 + 4] = s_relu;
  }
  bar();
  if (tid < 5) {
    float s = 0.f;
    for (int w = 0; w < NW; ++w) s += LP[w * 8 + tid];
    __hip_atomic_store((unsigned*)(a.partials + blk * 8 + tid), __builtin_bit_cast(unsigned, s), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if (CVAE_DIAG_STAMPS) lbar();  // the last stamp (thread 0, after the final barrier) before it is read
  if (CVAE_DIAG_STAMPS && a.stamps && tid < 64)
    gst<unsigned long long>(a.stamps + blk * 64 + tid, tid < stamp_i ? STAMPS[tid] : 0ull);
}

// BASELINE configs[0] / Training_VAE.py:274-282: seq_len 10, dim 3
using Cfg1 = Arch<10, 3>;
#ifndef CVAE_F32_RING
#define CVAE_F32_RING 16
#endif
// the largest batch the 4-row form serves by default (CVAE_F32_R4_MAX_BATCH overrides at run time)
#ifndef CVAE_F32_R4_MAX
#define CVAE_F32_R4_MAX 1024
#endif

// RR rows per workgroup (16, or 4: the 4x4x1_16b form for small batches, cvae_capi.hip f32c_rows)
// spread < 8: the row tiles on XCDs 0 .. spread-1 only (the grid is 8/spread times the tiles; block b
// runs on XCD b % 8, the others exit at once), so fewer L2s fetch the weight stream
template <class A, int RR>
__global__ __launch_bounds__(NT) void f32chain_kernel(char* arena, const void* x, const int64_t* idx, int Bp,
                                                      int batch, uint64_t* ctr, RowArgs a, int spread) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int blk = blockIdx.x;
  if (spread < 8) {
    const int xcd = blockIdx.x & 7;
    if (xcd >= spread) return;
    blk = (blockIdx.x >> 3) * spread + xcd;
  }
  RowArgs ra = a;
  ra.x = x;
  ra.idx = idx;
  ra.batch = batch;
  ra.ctr = ctr;
  f32_body<A, CVAE_F32_RING, RR>(arena, Bp, ra, smem, blk);
}

}  // namespace f32c
