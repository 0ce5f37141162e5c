// cvae_widechain.h — the bf16 training row chain specialised for BASELINE cfg5's wide shape
// (Training_VAE.py:118-167 widened: latent_dim 512, 8 encoder + 8 decoder Linears, seq_len 200;
// hidden_dim 128).
//
// Same work and the same arena outputs as rowchain_kernel<bf16, R, RC_TRAIN> (relative transform,
// forward, reparameterisation, conditional_vae_loss and dL/drecon, every dX; the feature-major
// xT/gT arena rows the dW kernel reduces), for one 16-row batch tile per workgroup.  The generic
// interpreter runs this shape with 8-row tiles (its tile state does not fit 16 rows of LDS) and
// is VALU/SALU-issue bound (38 VALU per MFMA at cfg5, profiles/r01i_wide_pmc_sq2.txt).  Here:
//  * UN-SWAPPED MFMA over feature-major LDS images (as cvae_fastchain.h): a lane's accumulator is
//    4 batch rows of ONE feature, so a ReLU mask is a 4-bit nibble of that lane — the 17 masks of
//    the chain live in 3 VGPRs, not in LDS — and the forward lane that produced a feature is the
//    backward lane that masks its gradient;
//  * mu, logvar and eps of the reparameterisation stay in the registers of the lanes that made
//    them (the fc n-tiles of wave w are mu tiles w, w+8, .. and logvar tiles Z/16 + w, ..; the
//    decoder-L0 backward hands wave w exactly the dz tiles of those latents), so nothing of the
//    R x Z latent state goes through LDS (3 x 32 KB at 16 rows);
//  * ONE WEIGHT STREAM per wave: the 397 fragments (1 KB each) the wave multiplies over the whole
//    chain, in consumption order, flow through a P-deep register ring — the fragment P items
//    ahead is issued as each one is consumed, across step boundaries, so the per-CU L2 stream
//    (3.2 MB per workgroup per step) never drains at a barrier.  Every index is compile-time
//    (sfor below): the ring is registers, not scratch;
//  * LDS 124 KB: dead buffers of the forward pass (fc input, decoder input, the recon time
//    channel) hold dL/d[mu ‖ logvar] in the backward pass.
// Selected by the host (cvae_capi.hip plan_wide) for bf16 training at exactly the Arch shape; every
// other configuration runs the generic interpreter (CVAE_GENERIC=1 forces it).
#pragma once
#include <type_traits>
#include "cvae_fastchain.h"

namespace wchain {

using fchain::H;
using fchain::NT;
using fchain::NW;
using fchain::R;
using fchain::arena4;
using fchain::bf16x4;
using fchain::from_bf4;
using fchain::ioff;
using fchain::lbar;
using fchain::quad_t;
using fchain::to_bf4;
using fchain::xfrag;

// compile-time loop: f(integral_constant<int, i>) for i in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

template <int S_, int D_, int Z_, int NE_, int ND_>
struct Arch {
  static constexpr int S = S_, D = D_, Z = Z_, NE = NE_, ND = ND_, I = S_ * D_;
  static constexpr int NKI = (I + 31) / 32, Ip = 32 * NKI;
  static constexpr int NL = 3 + NE + ND, ZH = Z + H;
  static constexpr int LC0 = 0, LC1 = 1, LE0 = 2, LFC = 2 + NE, LD0 = 3 + NE, LDL = 2 + NE + ND;
  static constexpr int LE(int i) { return 2 + i; }
  static constexpr int LD(int i) { return 3 + NE + i; }
  static constexpr int Kp(int l) { return l == LC0 ? 32 : l == LE0 ? Ip : l == LFC ? 2 * H : l == LD0 ? ZH : H; }
  static constexpr int Np(int l) { return l == LFC ? 2 * Z : l == LDL ? Ip : H; }
  // ReLU masks (forward order): C0 C1 E0..E(NE-1) D0..D(ND-2)
  static constexpr int MC0 = 0, MC1 = 1;
  static constexpr int ME(int i) { return 2 + i; }
  static constexpr int MD(int i) { return 2 + NE + i; }
  static constexpr int NMASK = 2 + NE + ND - 1, NMW = (NMASK + 7) / 8;
  static_assert(Z % 128 == 0, "latent tiles: 8 waves x whole 16-feature tiles of mu and logvar");
  static_assert(I % 8 == 0 && D >= 3, "x rows load as 16-B vectors; channels 0..2 = t, x, y");
  // the arena as alloc_arena (cvae_capi.hip) lays it out, bf16 operands: byte offsets from its base
  static constexpr int64_t r256(int64_t b) { return (b + 255) / 256 * 256; }
  static constexpr int64_t wf(int l) {
    int64_t o = 0;
    for (int k = 0; k < l; ++k) o += 2 * r256(2LL * Np(k) * Kp(k));
    return o;
  }
  static constexpr int64_t wb(int l) { return wf(l) + r256(2LL * Np(l) * Kp(l)); }
  static constexpr int bias_off(int l) {
    int o = 0;
    for (int k = 0; k < l; ++k) o += Np(k);
    return o;
  }
  static constexpr int nbias = bias_off(NL);
  static constexpr int64_t bias_base = wf(NL);
  static constexpr int64_t act0 = bias_base + r256(4LL * nbias);
  static constexpr int64_t xrows(int l) {  // xT(l) = act0 + 2·Bp·xrows(l) (Bp % 32 == 0)
    int64_t o = 0;
    for (int k = 0; k < l; ++k) o += Kp(k) + Np(k);
    return o;
  }
  static constexpr int64_t grows(int l) { return xrows(l) + Kp(l); }
  // LDS (bytes).  U: fc input, decoder input and the recon time channel (fp32) in the forward
  // pass; dL/d[mu ‖ logvar] (the fc backward's input image) from the decoder-L0 backward on
  static constexpr int L_XIN = 0, L_CIN = L_XIN + Ip * 32, L_CB = L_CIN + 32 * 32, L_A0 = L_CB + H * 32,
                       L_A1 = L_A0 + H * 32, L_U = L_A1 + H * 32;
  static constexpr int L_HCAT = L_U, L_DCAT = L_HCAT + 2 * H * 32, L_RCH0 = L_DCAT + ZH * 32,
                       L_GD0 = L_RCH0 + S * R * 4, L_UEND = L_GD0 + S * R * 4, L_GFC = L_U;
  static_assert(2 * Z * 32 <= L_UEND - L_U, "the fc-backward image fits in the dead forward buffers");
  static constexpr int L_BIAS = L_UEND, L_PART = L_BIAS + nbias * 4, L_TOTAL = L_PART + NW * 8 * 4;
  static_assert(L_TOTAL <= 160 * 1024, "LDS");
};

// One GEMM of the chain as its weight stream sees it: the operand (layer, forward Wf / backward
// Wb), its K chunks KC, the n-tiles of the output (NTL) and this wave's share (TS slots: tile
// wave + 8·slot; a slot past NTL reloads the last tile and its result is dropped).
struct StepInfo {
  int layer, bwd, KC, TS, NTL;
};

template <class A>
struct Plan {
  static constexpr StepInfo step(int s) {
    int k = 0;
    if (s == k++) return {A::LC0, 0, 1, 1, H / 16};
    if (s == k++) return {A::LE0, 0, A::NKI, 1, H / 16};
    if (s == k++) return {A::LC1, 0, H / 32, 1, H / 16};
    for (int i = 1; i < A::NE; ++i)
      if (s == k++) return {A::LE(i), 0, H / 32, 1, H / 16};
    if (s == k++) return {A::LFC, 0, 2 * H / 32, A::Z / 64, A::Z / 8};
    if (s == k++) return {A::LD0, 0, A::ZH / 32, 1, H / 16};
    for (int i = 1; i < A::ND - 1; ++i)
      if (s == k++) return {A::LD(i), 0, H / 32, 1, H / 16};
    if (s == k++) return {A::LDL, 0, H / 32, (A::Ip / 16 + NW - 1) / NW, A::Ip / 16};
    if (s == k++) return {A::LDL, 1, A::NKI, 1, H / 16};
    for (int i = A::ND - 2; i >= 1; --i)
      if (s == k++) return {A::LD(i), 1, H / 32, 1, H / 16};
    if (s == k++) return {A::LD0, 1, H / 32, A::ZH / 128, A::ZH / 16};
    if (s == k++) return {A::LFC, 1, 2 * A::Z / 32, 2, 2 * H / 16};
    for (int i = A::NE - 1; i >= 1; --i)
      if (s == k++) return {A::LE(i), 1, H / 32, 1, H / 16};
    if (s == k++) return {A::LC1, 1, H / 32, 1, H / 16};
    return {-1, 0, 0, 0, 0};
  }
  static constexpr int nsteps() {
    int s = 0;
    while (step(s).layer >= 0) ++s;
    return s;
  }
  static constexpr int NS = nsteps();
  static constexpr int start(int s) {
    int g = 0;
    for (int k = 0; k < s; ++k) g += step(k).KC * step(k).TS;
    return g;
  }
  static constexpr int total = start(NS);
  static constexpr int step_of(int g) {
    int s = 0;
    while (s + 1 < NS && start(s + 1) <= g) ++s;
    return s;
  }
  // step indices of the special GEMMs
  static constexpr int sE0 = 1, sC1 = 2, sFC = 2 + A::NE, sD0 = sFC + 1, sDL = sFC + A::ND, sDLb = sDL + 1,
                       sD0b = sDLb + A::ND - 1, sFCb = sD0b + 1, sC1b = NS - 1;
  static_assert(step(sFC).layer == A::LFC && !step(sFC).bwd && step(sDL).layer == A::LDL && !step(sDL).bwd &&
                    step(sDLb).layer == A::LDL && step(sDLb).bwd && step(sD0b).layer == A::LD0 &&
                    step(sD0b).bwd && step(sFCb).layer == A::LFC && step(sFCb).bwd,
                "step plan");
};

template <int P>
struct Ring {
  bf16x8 r[P];
};

// stream item G of this wave → ring slot G % P (no-op past the end of the stream)
template <class A, int P, int G>
__device__ __forceinline__ void ring_load(Ring<P>& ring, const char* AR, int wave, int lane) {
  using PL = Plan<A>;
  if constexpr (G < PL::total) {
    constexpr int s = PL::step_of(G);
    constexpr StepInfo st = PL::step(s);
    constexpr int j = G - PL::start(s), kc = j / st.TS, slot = j % st.TS;
    constexpr int64_t base = st.bwd ? A::wb(st.layer) : A::wf(st.layer);
    int w = wave;
    asm volatile("" : "+s"(w));  // recomputed per item: hoisted, ~400 item addresses would be live SGPRs
    int t = w + NW * slot;
    if constexpr (NW * (slot + 1) > st.NTL) t = min(t, st.NTL - 1);
    ring.r[G % P] = CVAE_DIAG_NOWLOAD ? bf16x8{}
                                      : gld<bf16x8>(AR + base + (int64_t)(t * st.KC + kc) * 1024 + lane * 16);
  }
}

// acc[slot] = X·Wᵀ for this wave's n-tiles of step S: X chunk kc read once (two transposed LDS
// reads), multiplied by every slot's fragment; each consumed ring slot is refilled P items ahead
template <class A, int P, int S, int TS>
__device__ __forceinline__ void gemm(Ring<P>& ring, const __bf16* img, f32x4 (&acc)[TS], const char* AR, int wave,
                                     int lane) {
  using PL = Plan<A>;
  constexpr StepInfo st = PL::step(S);
  static_assert(st.TS == TS, "accumulator slots");
  constexpr int G0 = PL::start(S);
  sfor<0, TS>([&](auto t) { acc[decltype(t)::value] = f32x4{0.f, 0.f, 0.f, 0.f}; });
  bf16x8 xf = xfrag(img, 0);
  sfor<0, st.KC>([&](auto kc) {
    constexpr int c = decltype(kc)::value;
    // the next chunk's X fragment is read one chunk ahead
    const bf16x8 xn = c + 1 < st.KC ? xfrag(img, c + 1) : xf;
    sfor<0, TS>([&](auto t) {
      constexpr int u = decltype(t)::value, g = G0 + c * TS + u;
      acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, ring.r[g % P], acc[u], 0, 0, 0);
      // Program order MFMA(g) → refill(g + P): the empty volatile asm on the result is ordered
      // before the (volatile) address step of the refill.  Left alone, the scheduler issues a
      // step's refills first and sinks its MFMA chains, and every ring slot then needs a second
      // register (spills).
      asm volatile("" : "+v"(acc[u]));
      ring_load<A, P, g + P>(ring, AR, wave, lane);
    });
    xf = xn;
  });
}

// the first P items of the stream (prologue)
template <class A, int P>
__device__ __forceinline__ void ring_fill(Ring<P>& ring, const char* AR, int wave, int lane) {
  sfor<0, P>([&](auto g) { ring_load<A, P, decltype(g)::value>(ring, AR, wave, lane); });
}

template <class A, int P>
__device__ __forceinline__ void wide_body(char* const AR, const int Bp, const RowArgs& a, char* smem, int blk) {
  using PL = Plan<A>;
  constexpr int Ip = A::Ip, S = A::S, D = A::D, I = A::I, Z = A::Z, NE = A::NE, ND = A::ND;
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int n16 = lane & 15, q = lane >> 4;
  const int b0 = blk * R, nrows = max(0, min(R, a.batch - b0));
  __bf16* const XIN = (__bf16*)(smem + A::L_XIN);
  __bf16* const CIN = (__bf16*)(smem + A::L_CIN);
  __bf16* const CB = (__bf16*)(smem + A::L_CB);
  __bf16* const A0 = (__bf16*)(smem + A::L_A0);
  __bf16* const A1 = (__bf16*)(smem + A::L_A1);
  __bf16* const HCAT = (__bf16*)(smem + A::L_HCAT);
  __bf16* const DCAT = (__bf16*)(smem + A::L_DCAT);
  __bf16* const GFC = (__bf16*)(smem + A::L_GFC);
  float* const RCH0 = (float*)(smem + A::L_RCH0);
  float* const GD0 = (float*)(smem + A::L_GD0);
  float* const BIAS = (float*)(smem + A::L_BIAS);
  float* const PART = (float*)(smem + A::L_PART);
  // arena matrices: recomputed at each use from Bp (one SGPR) — kept, the ~36 64-bit pointers of
  // the chain would be live scalar registers for the whole kernel (SGPR spills)
  auto XT = [&](int l) {
    int bp = Bp;
    asm volatile("" : "+s"(bp));
    return (void*)(AR + A::act0 + 2 * (int64_t)bp * A::xrows(l));
  };
  auto GT = [&](int l) {
    int bp = Bp;
    asm volatile("" : "+s"(bp));
    return (void*)(AR + A::act0 + 2 * (int64_t)bp * A::grows(l));
  };
  auto bias = [&](int l, int f) { return BIAS[A::bias_off(l) + f]; };
  const int n = 16 * wave + n16;  // this lane's feature in the 128-wide layers (n-tile = wave)

  // ReLU masks: nibble m of this lane (feature n, rows 4q..4q+3) at bits 4(m % 8) of mk[m / 8]
  uint32_t mk[A::NMW];
#pragma unroll
  for (int i = 0; i < A::NMW; ++i) mk[i] = 0u;
  auto relu = [&](f32x4 acc, float b, auto m) {
    constexpr int M = decltype(m)::value;
    f32x4 y;
    uint32_t nib = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y[i] = fmaxf(acc[i] + b, 0.f);
      nib |= (y[i] > 0.f ? 1u : 0u) << i;
    }
    mk[M / 8] |= nib << (4 * (M % 8));
    // materialise the mask word now: left lazy, the compiler keeps the four activations of every
    // layer alive until the backward pass needs the bits (VGPR spills)
    asm volatile("" : "+v"(mk[M / 8]));
    return to_bf4(y);
  };
  auto masked = [&](f32x4 acc, auto m) {
    constexpr int M = decltype(m)::value;
    const uint32_t nib = mk[M / 8] >> (4 * (M % 8));
    f32x4 y;
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = (nib >> i) & 1u ? acc[i] : 0.f;
    return to_bf4(y);
  };
  // one round (one (feature, row quad) task per thread) of the arena copy of the XIN image
  auto copy_round = [&](int k, void* mat, int Kf) {
    int t = tid;
    asm volatile("" : "+v"(t));  // per-round addresses: hoisted, every round's would stay live
    const int e = k * NT + t;
    if (e < Ip * 4) arena4(mat, Kf, e >> 2, b0, e & 3, *(const bf16x4*)(XIN + ioff(e >> 2, e & 3)));
  };
  constexpr int NCOPY = (Ip * 4 + NT - 1) / NT;  // rounds of one XIN copy

  Ring<P> ring;
  float s_recon = 0.f, s_kl = 0.f, s_start = 0.f, s_t0 = 0.f, s_relu = 0.f;

  // ---- prologue: x tile (relative transform, Training_VAE.py:345-348), biases, LDS pads
  {
    constexpr int U = (R * A::NKI * 4 + NT - 1) / NT;  // 16-B vectors per thread
    constexpr int VPR = I / 8, NV = R * VPR;
    const int last = max(a.batch - 1, 0);
    const __bf16* xg = (const __bf16*)a.x;
    bf16x8 xv[U], x0[U];
    int64_t gr[U];
    int cc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // task v: vector c of row 4rq + (v & 3) — quads = 4 rows, same c
      const int v = min(u * NT + tid, NV - 1);
      const int w = v >> 2, rq = w / VPR, c = w - rq * VPR, row = 4 * rq + (v & 3);
      gr[u] = min(b0 + row, last);
      cc[u] = c;
    }
    if (a.idx) {
#pragma unroll
      for (int u = 0; u < U; ++u) gr[u] = gld<int64_t>(a.idx + gr[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xv[u] = gld<bf16x8>(xg + gr[u] * I + cc[u] * 8);
      x0[u] = gld<bf16x8>(xg + gr[u] * I);  // the row's start point x[:,0,1:3] (Training_VAE.py:345)
    }
    constexpr int NB4 = A::nbias / 4, UB = (NB4 + NT - 1) / NT;
    f32x4 bv[UB];
#pragma unroll
    for (int k = 0; k < UB; ++k) bv[k] = gld<f32x4>((const float*)(AR + A::bias_base) + 4 * min(k * NT + tid, NB4 - 1));
    // the weight stream queues behind the x tile and the biases (vmcnt retires in order)
    ring_fill<A, P>(ring, AR, wave, lane);
    if (a.ctr && blk == 0 && tid == 0) adam_precompute(a.ctr, a.lr, a.beta1, a.beta2, a.adam_pre);
    if (tid < 28 * 4) *(uint64_t*)(CIN + (4 + tid / 4) * 16 + 4 * (tid & 3)) = 0ull;
    if (tid < (Ip - I) * 4) *(uint64_t*)(XIN + (I + tid / 4) * 16 + 4 * (tid & 3)) = 0ull;
#pragma unroll
    for (int k = 0; k < UB; ++k)
      if (k * NT + tid < NB4) ((f32x4*)BIAS)[k * NT + tid] = bv[k];
    void* const xc0 = XT(A::LC0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = u * NT + tid;
      if (v < NV) {  // NV % 4 == 0: quads are whole
        const int w = v >> 2, rq = w / VPR, c = w - rq * VPR;
        const int qd = lane & 3, f0 = c * 8;
        const f32x4 xlo = quad_t(f32x4{(float)xv[u][0], (float)xv[u][1], (float)xv[u][2], (float)xv[u][3]});
        const f32x4 xhi = quad_t(f32x4{(float)xv[u][4], (float)xv[u][5], (float)xv[u][6], (float)xv[u][7]});
        const float s0 = (float)x0[u][1], s1 = (float)x0[u][2];
        const f32x4 S0 = fchain::quad_all(s0), S1 = fchain::quad_all(s1);
        const int fl = f0 + qd, fh = fl + 4;
        const int dl = fl % D, dh = fh % D;
        const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
        f32x4 rl = xlo - (dl == 1 ? S0 : dl == 2 ? S1 : zero);
        f32x4 rh = xhi - (dh == 1 ? S0 : dh == 2 ? S1 : zero);
        f32x4 cv = qd == 0 ? S0 : qd == 1 ? S1 : zero;
        if (nrows < R) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bool live = 4 * rq + i < nrows;
            rl[i] = live ? rl[i] : 0.f;
            rh[i] = live ? rh[i] : 0.f;
            cv[i] = live ? cv[i] : 0.f;
          }
        }
        *(bf16x4*)(XIN + ioff(fl, rq)) = to_bf4(rl);
        *(bf16x4*)(XIN + ioff(fh, rq)) = to_bf4(rh);
        if (c == 0) {
          const bf16x4 cs = to_bf4(cv);
          *(bf16x4*)(CIN + ioff(qd, rq)) = cs;
          arena4(xc0, A::Kp(A::LC0), qd, b0, rq, cs);
        }
      }
    }
  }
  lbar();

  const float Bf = (float)a.batch;
  const float inv_BSD = 1.f / (Bf * (float)(S * D)), inv_2B = 1.f / (2.f * Bf), inv_B = 1.f / Bf;
  const float inv_BS1 = S > 1 ? 1.f / (Bf * (float)(S - 1)) : 0.f, inv_BZ = 1.f / (Bf * (float)Z);
  const bool use_start = a.w_start > 0.f, use_time = a.w_time > 0.f;  // Training_VAE.py:247, :256

  // ================================================================ forward
  {  // C0 ‖ E0
    f32x4 acc[1];
    gemm<A, P, 0>(ring, CIN, acc, AR, wave, lane);
    const bf16x4 hc = relu(acc[0], bias(A::LC0, n), std::integral_constant<int, A::MC0>{});
    *(bf16x4*)(CB + ioff(n, q)) = hc;
    arena4(XT(A::LC1), A::Kp(A::LC1), n, b0, q, hc);
    gemm<A, P, PL::sE0>(ring, XIN, acc, AR, wave, lane);
    const bf16x4 he = relu(acc[0], bias(A::LE0, n), std::integral_constant<int, A::ME(0)>{});
    *(bf16x4*)(A0 + ioff(n, q)) = he;
    arena4(XT(A::LE(1)), A::Kp(A::LE(1)), n, b0, q, he);
  }
  lbar();
  {  // C1 ‖ E1: h_c goes to both concatenations (fc input at H+n, decoder input at Z+n)
    f32x4 acc[1];
    gemm<A, P, PL::sC1>(ring, CB, acc, AR, wave, lane);
    const bf16x4 hc = relu(acc[0], bias(A::LC1, n), std::integral_constant<int, A::MC1>{});
    *(bf16x4*)(HCAT + ioff(H + n, q)) = hc;
    *(bf16x4*)(DCAT + ioff(Z + n, q)) = hc;
    arena4(XT(A::LFC), A::Kp(A::LFC), H + n, b0, q, hc);
    arena4(XT(A::LD0), A::Kp(A::LD0), Z + n, b0, q, hc);
  }
  // encoder layers 1 .. NE-1 (input image: E(i-1)'s output, A0 for odd i); the last → h_traj
  sfor<1, NE>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    if constexpr (i > 1) lbar();
    f32x4 acc[1];
    gemm<A, P, PL::sC1 + i>(ring, (i & 1) ? A0 : A1, acc, AR, wave, lane);
    const bf16x4 he = relu(acc[0], bias(A::LE(i), n), std::integral_constant<int, A::ME(i)>{});
    if constexpr (i == NE - 1) {
      *(bf16x4*)(HCAT + ioff(n, q)) = he;
      arena4(XT(A::LFC), A::Kp(A::LFC), n, b0, q, he);
    } else {
      *(bf16x4*)(((i & 1) ? A1 : A0) + ioff(n, q)) = he;
      arena4(XT(A::LE(i + 1)), A::Kp(A::LE(i + 1)), n, b0, q, he);
    }
    // the x_rel tile → xT(E0): spread over the encoder steps, done before the loss overwrites XIN
    if constexpr (i <= 5) {
#pragma unroll
      for (int k = 2 * (i - 1); k < 2 * i && k < NCOPY; ++k) copy_round(k, XT(A::LE0), A::Kp(A::LE0));
    }
  });
  static_assert(NCOPY <= 10 && NE >= 6, "the x_rel copy needs 5 encoder steps");
  lbar();
  // fc_mu ‖ fc_logvar (:195-196) + reparameterize (:199-206) + KL terms (:243): slot k < Z/128 is
  // mu tile wave + 8k, slot k + Z/128 the logvar tile of the same latents
  constexpr int NZT = Z / 128;
  f32x4 mu[NZT], lv[NZT], ep[NZT];
  {
    f32x4 acc[2 * NZT];
    gemm<A, P, PL::sFC>(ring, HCAT, acc, AR, wave, lane);
    const uint64_t off = rng_offset(a);
    const int rowq = 4 * q + (n16 & 3);  // the row this lane draws (4 latents) before the quad transpose
#pragma unroll
    for (int k = 0; k < NZT; ++k) {
      const int j = 16 * (wave + NW * k) + n16, j0 = 16 * (wave + NW * k) + 4 * (n16 >> 2);
      f32x4 e = {0.f, 0.f, 0.f, 0.f};
      if (rowq < nrows)  // Philox keyed by the global row (data parallelism: eps_row0 = the rank's first row)
        e = a.eps ? gld<f32x4>(a.eps + (size_t)(b0 + rowq) * Z + j0)
                  : philox_normal4(a.seed, off, (uint32_t)(a.eps_row0 + b0 + rowq), (uint32_t)j0);
      ep[k] = quad_t(e);  // eps of latent j, rows 4q .. 4q+3
      const float bm = bias(A::LFC, j), bl = bias(A::LFC, Z + j);
      f32x4 z;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        mu[k][i] = acc[k][i] + bm;
        lv[k][i] = acc[NZT + k][i] + bl;
        const float sd = __expf(0.5f * lv[k][i]);
        z[i] = mu[k][i] + ep[k][i] * sd;
        if (4 * q + i < nrows) s_kl += 1.f + lv[k][i] - mu[k][i] * mu[k][i] - __expf(lv[k][i]);
      }
      const bf16x4 zh = to_bf4(z);
      *(bf16x4*)(DCAT + ioff(j, q)) = zh;
      arena4(XT(A::LD0), A::Kp(A::LD0), j, b0, q, zh);
    }
  }
  lbar();
  {  // D0 → A0
    f32x4 acc[1];
    gemm<A, P, PL::sD0>(ring, DCAT, acc, AR, wave, lane);
    const bf16x4 h = relu(acc[0], bias(A::LD0, n), std::integral_constant<int, A::MD(0)>{});
    *(bf16x4*)(A0 + ioff(n, q)) = h;
    arena4(XT(A::LD(1)), A::Kp(A::LD(1)), n, b0, q, h);
  }
  // decoder layers 1 .. ND-2 (input: D(i-1)'s output, A0 for odd i)
  sfor<1, ND - 1>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    lbar();
    f32x4 acc[1];
    gemm<A, P, PL::sD0 + i>(ring, (i & 1) ? A0 : A1, acc, AR, wave, lane);
    const bf16x4 h = relu(acc[0], bias(A::LD(i), n), std::integral_constant<int, A::MD(i)>{});
    *(bf16x4*)(((i & 1) ? A1 : A0) + ioff(n, q)) = h;
    arena4(XT(A::LD(i + 1)), A::Kp(A::LD(i + 1)), n, b0, q, h);
  });
  lbar();
  __bf16* const DLIN = ((ND - 2) & 1) ? A1 : A0;  // input image of the last decoder layer
  {  // last decoder layer + conditional_vae_loss (:229-268) + dL/drecon, over x_rel in place
    constexpr StepInfo st = PL::step(PL::sDL);
    constexpr int G3 = st.TS, NG3 = st.NTL;
    auto has = [&](int g) { return NW * (g + 1) <= NG3 || wave + NW * g < NG3; };
    f32x4 accs[G3];
    gemm<A, P, PL::sDL>(ring, DLIN, accs, AR, wave, lane);
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const float cr = a.w_recon * 2.f;
    f32x2 sr2 = {0.f, 0.f};
#pragma unroll
    for (int g = 0; g < G3; ++g) {
      if (!has(g)) continue;
      const int t = wave + NW * g;
      const f32x4 acc = accs[g];
      const int f = 16 * t + n16;
      f32x4 gi = {0.f, 0.f, 0.f, 0.f};
      if (f < I) {
        const float b = bias(A::LDL, f);
        const f32x4 xr = from_bf4(*(const bf16x4*)(XIN + ioff(f, q)));
        const int s = f / D, d = f - s * D;
        const f32x2 r01 = f32x2{acc[0], acc[1]} + b, r23 = f32x2{acc[2], acc[3]} + b;
        f32x2 d01 = r01 - f32x2{xr[0], xr[1]}, d23 = r23 - f32x2{xr[2], xr[3]};
        if (nrows < R) {
          d01[0] = 4 * q + 0 < nrows ? d01[0] : 0.f;
          d01[1] = 4 * q + 1 < nrows ? d01[1] : 0.f;
          d23[0] = 4 * q + 2 < nrows ? d23[0] : 0.f;
          d23[1] = 4 * q + 3 < nrows ? d23[1] : 0.f;
        }
        sr2 += d01 * d01;
        sr2 += d23 * d23;
        const f32x2 g01 = d01 * cr * inv_BSD, g23 = d23 * cr * inv_BSD;  // w_recon·2·diff / (B·S·D)
        gi = f32x4{g01[0], g01[1], g23[0], g23[1]};
        const f32x4 r = {r01[0], r01[1], r23[0], r23[1]};
        if (16 * t < D) {  // wave-uniform: only these n-tiles hold timestep-0 features
          const f32x4 df = {d01[0], d01[1], d23[0], d23[1]};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (4 * q + i >= nrows) continue;
            if (s == 0 && (d == 1 || d == 2) && use_start) {
              s_start += df[i] * df[i];
              gi[i] += a.w_start * 2.f * df[i] * inv_2B;
            }
            if (d == 0 && s == 0 && use_time) {
              s_t0 += r[i] * r[i];
              gi[i] += a.w_time * 2.f * r[i] * inv_B;
            }
          }
        }
        if (d == 0) {
          *(f32x4*)(RCH0 + s * R + 4 * q) = r;
          *(f32x4*)(GD0 + s * R + 4 * q) = gi;
        }
      }
      *(bf16x4*)(XIN + ioff(f, q)) = to_bf4(gi);  // pad features f >= I: 0
    }
    s_recon += sr2[0] + sr2[1];
  }
  lbar();
  // time-monotonicity term relu(r_s − r_{s+1}) (:261-262, ReLU'(0) = 0) into the time channel of
  // dL/drecon: one task per (timestep, row quad)
  {
    const float wt = a.w_time * inv_BS1;
    for (int e = tid; e < S * 4; e += NT) {
      const int s = e >> 2, qq = e & 3, f = s * D;
      f32x4 gv = *(const f32x4*)(GD0 + s * R + 4 * qq);
      if (use_time) {
        const f32x4 rs = *(const f32x4*)(RCH0 + s * R + 4 * qq);
        const f32x4 rn = *(const f32x4*)(RCH0 + min(s + 1, S - 1) * R + 4 * qq);
        const f32x4 rp = *(const f32x4*)(RCH0 + max(s - 1, 0) * R + 4 * qq);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool live = 4 * qq + i < nrows;
          const float u1 = rs[i] - rn[i], u0 = rp[i] - rs[i];  // 0 at the sequence ends
          if (live && u1 > 0.f) {
            gv[i] += wt;
            s_relu += u1;
          }
          if (live && u0 > 0.f) gv[i] -= wt;
        }
      }
      *(bf16x4*)(XIN + ioff(f, qq)) = to_bf4(gv);
    }
  }
  lbar();

  // ================================================================ backward
  {  // last decoder layer ᵀ: dL/d h_D(ND-2) = GL · W_DL, ReLU mask of D(ND-2) → A0
    f32x4 acc[1];
    gemm<A, P, PL::sDLb>(ring, XIN, acc, AR, wave, lane);
    const bf16x4 h = masked(acc[0], std::integral_constant<int, A::MD(ND - 2)>{});
    *(bf16x4*)(A0 + ioff(n, q)) = h;
    arena4(GT(A::LD(ND - 2)), A::Np(A::LD(ND - 2)), n, b0, q, h);
  }
  // dL/drecon → gT(DL), spread over the decoder backward steps
  copy_round(0, GT(A::LDL), A::Np(A::LDL));
  copy_round(1, GT(A::LDL), A::Np(A::LDL));
  static_assert(ND >= 6, "the dL/drecon copy needs 5 decoder backward steps");
  // D(i)ᵀ for i = ND-2 .. 1: input = the gradient image of D(i)'s output, mask of D(i-1)
  sfor<1, ND - 1>([&](auto kk) {
    constexpr int k = decltype(kk)::value, i = ND - 1 - k;  // k-th decoder backward step after DLᵀ
    lbar();
    f32x4 acc[1];
    gemm<A, P, PL::sDLb + k>(ring, (k & 1) ? A0 : A1, acc, AR, wave, lane);
    const bf16x4 h = masked(acc[0], std::integral_constant<int, A::MD(i - 1)>{});
    *(bf16x4*)(((k & 1) ? A1 : A0) + ioff(n, q)) = h;
    arena4(GT(A::LD(i - 1)), A::Np(A::LD(i - 1)), n, b0, q, h);
    if constexpr (k <= 4) {
#pragma unroll
      for (int r = 2 * k; r < 2 * k + 2 && r < NCOPY; ++r) copy_round(r, GT(A::LDL), A::Np(A::LDL));
    }
  });
  lbar();
  // D0ᵀ: [dz ‖ dh_c(decoder share)]; dz → KL/reparameterisation backward → dL/d[mu ‖ logvar]
  __bf16* const D0IN = ((ND - 2) & 1) ? A1 : A0;  // gradient image of D0's output
  f32x4 dhc2;
  {
    f32x4 acc[NZT + 1];
    gemm<A, P, PL::sD0b>(ring, D0IN, acc, AR, wave, lane);
#pragma unroll
    for (int k = 0; k < NZT; ++k) {
      const int j = 16 * (wave + NW * k) + n16;
      f32x4 gm, gl;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool live = 4 * q + i < nrows;
        const float sd = __expf(0.5f * lv[k][i]);
        gm[i] = live ? a.w_kld * mu[k][i] * inv_BZ + acc[k][i] : 0.f;
        gl[i] = live ? a.w_kld * 0.5f * (__expf(lv[k][i]) - 1.f) * inv_BZ + acc[k][i] * ep[k][i] * 0.5f * sd : 0.f;
      }
      const bf16x4 hm = to_bf4(gm), hl = to_bf4(gl);
      *(bf16x4*)(GFC + ioff(j, q)) = hm;
      *(bf16x4*)(GFC + ioff(Z + j, q)) = hl;
      arena4(GT(A::LFC), A::Np(A::LFC), j, b0, q, hm);
      arena4(GT(A::LFC), A::Np(A::LFC), Z + j, b0, q, hl);
    }
    dhc2 = acc[NZT];  // feature n of dh_c: the lane that masks it in the fc backward
  }
  lbar();
  {  // fcᵀ: dh = G_fc · W_fc → h_traj gradient (mask E(NE-1)) and h_c gradient (+ decoder share, mask C1)
    f32x4 acc[2];
    gemm<A, P, PL::sFCb>(ring, GFC, acc, AR, wave, lane);
    const bf16x4 ht = masked(acc[0], std::integral_constant<int, A::ME(NE - 1)>{});
    *(bf16x4*)(A0 + ioff(n, q)) = ht;
    arena4(GT(A::LE(NE - 1)), A::Np(A::LE(NE - 1)), n, b0, q, ht);
    const bf16x4 hc = masked(acc[1] + dhc2, std::integral_constant<int, A::MC1>{});
    *(bf16x4*)(CB + ioff(n, q)) = hc;
    arena4(GT(A::LC1), A::Np(A::LC1), n, b0, q, hc);
  }
  // E(i)ᵀ for i = NE-1 .. 2 (input: gradient image of E(i)'s output), mask of E(i-1)
  sfor<0, NE - 2>([&](auto kk) {
    constexpr int k = decltype(kk)::value, i = NE - 1 - k;
    lbar();
    f32x4 acc[1];
    gemm<A, P, PL::sFCb + 1 + k>(ring, (k & 1) ? A1 : A0, acc, AR, wave, lane);
    const bf16x4 h = masked(acc[0], std::integral_constant<int, A::ME(i - 1)>{});
    *(bf16x4*)(((k & 1) ? A0 : A1) + ioff(n, q)) = h;
    arena4(GT(A::LE(i - 1)), A::Np(A::LE(i - 1)), n, b0, q, h);
  });
  lbar();
  {  // E1ᵀ ‖ C1ᵀ: the last two gradients only feed the dW kernel
    f32x4 acc[1];
    gemm<A, P, PL::sC1b - 1>(ring, ((NE - 2) & 1) ? A1 : A0, acc, AR, wave, lane);
    arena4(GT(A::LE0), A::Np(A::LE0), n, b0, q, masked(acc[0], std::integral_constant<int, A::ME(0)>{}));
    gemm<A, P, PL::sC1b>(ring, CB, acc, AR, wave, lane);
    arena4(GT(A::LC0), A::Np(A::LC0), n, b0, q, masked(acc[0], std::integral_constant<int, A::MC0>{}));
  }

  // ---- loss partial sums (deterministic order)
  s_recon = wave_sum(s_recon);
  s_kl = wave_sum(s_kl);
  s_start = wave_sum(s_start);
  s_t0 = wave_sum(s_t0);
  s_relu = wave_sum(s_relu);
  if (lane == 0) {
    PART[wave * 8 + 0] = s_recon;
    PART[wave * 8 + 1] = s_kl;
    PART[wave * 8 + 2] = s_start;
    PART[wave * 8 + 3] = s_t0;
    PART[wave * 8 + 4] = s_relu;
  }
  lbar();
  if (tid < 5) {
    float s = 0.f;
    for (int w = 0; w < NW; ++w) s += PART[w * 8 + tid];
    gst<float>(a.partials + blk * 8 + tid, s);
  }
}

// BASELINE cfg5: S=200, D=6, latent 512, 8 + 8 layers (hidden 128)
using Cfg5 = Arch<200, 6, 512, 8, 8>;
#ifndef CVAE_WIDE_RING
#define CVAE_WIDE_RING 12
#endif
constexpr int RING = CVAE_WIDE_RING;

template <class A>
__global__ __launch_bounds__(NT) void widechain_kernel(char* arena, const void* x, const int64_t* idx, int Bp,
                                                       int batch, RowArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  RowArgs ra = a;
  ra.x = x;
  ra.idx = idx;
  ra.batch = batch;
  wide_body<A, RING>(arena, Bp, ra, smem, blockIdx.x);
}

}  // namespace wchain
