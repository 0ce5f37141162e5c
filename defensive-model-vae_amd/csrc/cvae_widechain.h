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

// F8_: the CVAE_FP8 form — every forward GEMM whose padded K is a multiple of 64 multiplies e4m3
// activations by e4m3(s·W) fragments (half the weight stream); backward GEMMs stay bf16.
// CLS_: BASELINE cfg4's scenario-class embedding (a build-side extension of Training_VAE.py:193,
// :214): e = table[class] (class_dim <= CLS_EMAX features, n_classes <= 32) joins both
// concatenations, [h_traj ‖ h_c ‖ e] and [z ‖ h_c ‖ e]; the table is the last layer (LCE, one-hot
// input, no bias, no activation).  Its padded dims do not depend on class_dim within that bound, so
// one instantiation serves every class_dim the host accepts (plan_ring_cls).
// MXB_ (with F8_): the large dX GEMMs in e4m3 with MX block scales (f8b below); false keeps every
// backward GEMM bf16 — the creation-time fallback CVAE_FP8_DX=bf16 (cvae_capi.hip build_plan).
template <int S_, int D_, int Z_, int NE_, int ND_, bool F8_ = false, bool CLS_ = false, bool MXB_ = F8_>
struct Arch {
  static constexpr int S = S_, D = D_, Z = Z_, NE = NE_, ND = ND_, I = S_ * D_;
  static constexpr bool F8 = F8_, CLS = CLS_, MXB = MXB_ && F8_;
  static constexpr int CLS_EMAX = 24, CLS_NMAX = 32;
  static constexpr int NKI = (I + 31) / 32, Ip = 32 * NKI;
  static constexpr int NL = 3 + NE + ND + (CLS_ ? 1 : 0), ZH = Z + H;
  // SZ: a latent of one 16-feature tile of mu ‖ logvar (the reference architecture, latent 8): fc is
  // one n-tile, split over the waves by K; dz and dh_c of the decoder-L0 backward are not tile-aligned
  static constexpr bool SZ = 2 * Z == 16;
  static constexpr int r32(int v) { return (v + 31) / 32 * 32; }
  static constexpr int LC0 = 0, LC1 = 1, LE0 = 2, LFC = 2 + NE, LD0 = 3 + NE, LDL = 2 + NE + ND,
                       LCE = CLS_ ? 3 + NE + ND : -1;
  static constexpr int LE(int i) { return 2 + i; }
  static constexpr int LD(int i) { return 3 + NE + i; }
  static constexpr int Kp(int l) {
    return l == LC0 ? 32 : l == LE0 ? Ip : l == LFC ? (CLS ? r32(2 * H + CLS_EMAX) : 2 * H)
         : l == LD0 ? r32(ZH + (CLS ? CLS_EMAX : 0)) : l == LCE ? CLS_NMAX : H;
  }
  static constexpr int Np(int l) { return l == LFC ? r32(2 * Z) : l == LDL ? Ip : l == LCE ? r32(CLS_EMAX) : H; }
  // fc's K chunks (32 wide): 2H/32, and one more for the class embedding
  static constexpr int FC_KCH = (CLS ? r32(2 * H + CLS_EMAX) : 2 * H) / 32;
  // ReLU masks (forward order): C0 C1 E0..E(NE-1) D0..D(ND-2)
  static constexpr int MC0 = 0, MC1 = 1;
  static constexpr int ME(int i) { return 2 + i; }
  static constexpr int MD(int i) { return 2 + NE + i; }
  static constexpr int NMASK = 2 + NE + ND - 1, NMW = (NMASK + 7) / 8;
  static_assert(Z % 128 == 0 || SZ, "latent tiles: 8 waves x whole 16-feature tiles of mu and logvar, or one tile");
  static_assert(!SZ || (FC_KCH >= NW && FC_KCH <= 2 * NW), "small latent: fc's K chunks split over the waves");
  static_assert(!CLS || (SZ && r32(2 * H + CLS_EMAX) == r32(2 * H + 4) && r32(ZH + CLS_EMAX) == r32(ZH + 4)),
                "class embedding: padded fc / decoder-input K independent of class_dim in [4, CLS_EMAX]");
  static_assert(I % 8 == 0 && D >= 3, "x rows load as 16-B vectors; channels 0..2 = t, x, y");
  // the layers the fp8 form runs in e4m3 (cvae_capi.hip build_plan: padded K % 64 == 0)
  static constexpr bool f8(int l) { return F8 && Kp(l) % 64 == 0; }
  // the layers whose dX GEMM the fp8 form runs in e4m3 (cvae_capi.hip build_plan, LayerDev::f8b):
  // e4m3 forward operand, backward K (= Np) pairing up, a dX at all (not C0 / E0), and large enough
  // for the halved stream to matter — at cfg5 the last decoder layer, decoder L0 and fc
  static constexpr bool f8b(int l) {
    return MXB && f8(l) && Np(l) % 64 == 0 && l != LC0 && l != LE0 && (Np(l) >= 512 || Kp(l) >= 512);
  }
  // the arena as alloc_arena (cvae_capi.hip) lays it out, bf16 operands: byte offsets from its base;
  // an e4m3 layer's Wf region starts with its 256-B F8Scale header
  static constexpr int64_t r256(int64_t b) { return (b + 255) / 256 * 256; }
  static constexpr int64_t hdr(int l) { return f8(l) ? (int64_t)sizeof(F8Scale) : 0; }
  // per layer: Wf (bf16, or e4m3 behind its F8Scale header), Wb (bf16), and where f8b: Wb8 (e4m3)
  static constexpr int64_t region(int l) {
    int64_t o = 0;
    for (int k = 0; k < l; ++k)
      o += r256(2LL * Np(k) * Kp(k) + hdr(k)) + r256(2LL * Np(k) * Kp(k)) + (f8b(k) ? r256(1LL * Np(k) * Kp(k)) : 0);
    return o;
  }
  static constexpr int64_t wf(int l) { return region(l) + hdr(l); }
  static constexpr int64_t wb(int l) { return region(l) + r256(2LL * Np(l) * Kp(l) + hdr(l)); }
  static constexpr int64_t wb8(int l) { return wb(l) + r256(2LL * Np(l) * Kp(l)); }
  static constexpr int bias_off(int l) {
    int o = 0;
    for (int k = 0; k < l; ++k) o += Np(k);
    return o;
  }
  static constexpr int nbias = bias_off(NL);
  static constexpr int64_t bias_base = region(NL);
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
  static constexpr int L_HCAT = L_U, L_DCAT = L_HCAT + Kp(LFC) * 32, L_RCH0 = L_DCAT + Kp(LD0) * 32,
                       L_GD0 = L_RCH0 + S * R * 4, L_UEND = L_GD0 + S * R * 4, L_GFC = L_U;
  static_assert(Np(LFC) * 32 <= L_UEND - L_U, "the fc-backward image fits in the dead forward buffers");
  // SZ only: fc's per-wave partial sums (fp32 [wave][feature][row], in A0 ‖ A1, dead at fc) and the
  // decoder share of dh_c (fp32 [c][row], behind the fc-backward image in the dead U region)
  static constexpr int L_PFC = L_A0, L_DHC2 = L_GFC + Np(LFC) * 32;
  static_assert(!SZ || (NW * 16 * R * 4 <= 2 * H * 32 && L_DHC2 + H * R * 4 <= L_UEND), "SZ buffers");
  // F8: e4m3 images (fragment order, 16 B per feature, img8) beside the bf16 ones of every input of
  // an e4m3 GEMM: the condition h (C1's input), the hidden ping-pong pair, the fc input; the
  // encoder-L1 input (converted after C0, read by E0) and later the decoder input share the recon
  // time channel's buffers (dead until the last decoder layer)
  static constexpr int F8B = F8 ? 16 : 0;
  static constexpr int L_CB8 = L_UEND, L_A08 = L_CB8 + H * F8B, L_A18 = L_A08 + H * F8B,
                       L_HCAT8 = L_A18 + H * F8B, L_X8 = L_RCH0, L_DCAT8 = L_RCH0;
  static_assert(!F8 || (Ip * 16 <= 2 * S * R * 4 && Kp(LD0) * 16 <= 2 * S * R * 4 && Ip % 64 == 0 &&
                        Kp(LD0) % 64 == 0),
                "fp8 images");
  static constexpr int L_INVS = L_HCAT8 + 2 * H * F8B;  // 1/s of every layer (1 where bf16)
  // the e4m3 twin of the bf16 image at LDS offset L (compile-time at every use: a pointer-valued
  // mapping became a lookup table in scratch memory)
  static constexpr int twin_off(int L) {
    return L == L_A0 ? L_A08 : L == L_A1 ? L_A18 : L == L_CB ? L_CB8 : L == L_HCAT ? L_HCAT8
         : L == L_DCAT ? L_DCAT8 : L == L_XIN ? L_X8 : -1;
  }
  // CLS: the one-hot class image (xT(LCE), 32 features), the de image (gT(LCE)), the decoder's
  // share of de (fp32 [feature][row]) and the rows' class ids
  static constexpr int L_CLS1H = L_INVS + (F8 ? 32 * 4 : 0), L_GCE = L_CLS1H + (CLS ? CLS_NMAX * 32 : 0),
                       L_DCE2 = L_GCE + (CLS ? Np(LCE) * 32 : 0), L_CLSID = L_DCE2 + (CLS ? CLS_EMAX * R * 4 : 0),
                       L_CTAB = L_CLSID + (CLS ? R * 4 : 0);  // the table's operand copy (Wf(LCE), 2 KB)
  static constexpr int L_BIAS = L_CTAB + (CLS ? 2 * Np(LCE) * Kp(LCE) : 0), L_PART = L_BIAS + nbias * 4,
                       L_STAMPS = L_PART + NW * 8 * 4, L_TOTAL = L_STAMPS + (CVAE_DIAG_STAMPS ? 64 * 8 : 0);
  static_assert(NL <= 32, "1/s table");
  static_assert(L_TOTAL <= 160 * 1024, "LDS");
};

// One GEMM of the chain as its weight stream sees it: the operand (layer, forward Wf / backward
// Wb), its K chunks KC, the n-tiles of the output (NTL) and this wave's share (TS slots: tile
// wave + 8·slot; a slot past NTL reloads the last tile and its result is dropped).
// GRP > 0: the slots run in TS/GRP groups of GRP (group p = slots p, p + TS/GRP, ..), each group's
// whole K before the next (its epilogue then overlaps the next group's stream; the X operand, KC
// chunks, is read once and held); GRP = 0: K-chunk-major over all slots (X streamed).
// KS = 1: one n-tile whose K chunks are split over the waves (chunk = wave; one item per wave), the
// partial sums reduced through LDS by the step's epilogue.
// F8 = 1: an e4m3 forward GEMM — KC counts 64-wide K pairs (one 16-B fragment each).
struct StepInfo {
  int layer, bwd, KC, TS, NTL, GRP, KS, F8;
};

template <class A>
struct Plan {
  static constexpr StepInfo step(int s) {
    StepInfo st = step0(s);
    if (st.layer >= 0 && !st.bwd && A::f8(st.layer)) {  // e4m3: K pairs
      st.KC = st.KS ? st.KC : st.KC / 2;
      st.F8 = 1;
    }
    if (st.layer >= 0 && st.bwd && A::f8b(st.layer)) {  // e4m3 dX with MX row-block scales (gemm_mxb)
      st.KC = (st.KC + 1) / 2;
      st.F8 = 2;
    }
    return st;
  }
  static constexpr StepInfo step0(int s) {
    int k = 0;
    if (s == k++) return {A::LC0, 0, 1, 1, H / 16};
    if (s == k++) return {A::LE0, 0, A::NKI, 1, H / 16};
    if (s == k++) return {A::LC1, 0, H / 32, 1, H / 16};
    for (int i = 1; i < A::NE; ++i)
      if (s == k++) return {A::LE(i), 0, H / 32, 1, H / 16};
    if (s == k++)  // SZ: K chunks wave, wave + 8 (KC items per wave; a chunk past FC_KCH is skipped)
      return A::SZ ? StepInfo{A::LFC, 0, (A::FC_KCH + NW - 1) / NW, 1, 1, 0, 1}
                   : StepInfo{A::LFC, 0, 2 * H / 32, A::Z / 64, A::Z / 8, 2};
    if (s == k++) return {A::LD0, 0, A::Kp(A::LD0) / 32, 1, H / 16};
    for (int i = 1; i < A::ND - 1; ++i)
      if (s == k++) return {A::LD(i), 0, H / 32, 1, H / 16};
    if (s == k++) return {A::LDL, 0, H / 32, (A::Ip / 16 + NW - 1) / NW, A::Ip / 16, 1};
    if (s == k++) return {A::LDL, 1, A::NKI, 1, H / 16};
    for (int i = A::ND - 2; i >= 1; --i)
      if (s == k++) return {A::LD(i), 1, H / 32, 1, H / 16};
    if (s == k++) return {A::LD0, 1, H / 32, (A::Kp(A::LD0) / 16 + NW - 1) / NW, A::Kp(A::LD0) / 16};
    if (s == k++) return {A::LFC, 1, A::Np(A::LFC) / 32, (A::Kp(A::LFC) / 16 + NW - 1) / NW, A::Kp(A::LFC) / 16};
    for (int i = A::NE - 1; i >= 1; --i)
      if (s == k++) return {A::LE(i), 1, H / 32, 1, H / 16};
    if (s == k++) return {A::LC1, 1, H / 32, 1, H / 16};
    return {-1, 0, 0, 0, 0, 0, 0, 0};
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

#ifndef CVAE_DIAG_NOPHILOX
#define CVAE_DIAG_NOPHILOX 0  // timing only: eps = 0 without the Philox draws
#endif
#ifndef CVAE_DIAG_NOADAMPRE
#define CVAE_DIAG_NOADAMPRE 0  // timing only: no Adam-scalar precompute in block 0
#endif
template <int P>
struct Ring {
  bf16x8 r[P];
};

// Measured choices of the prologue and the stream, kept as constants (the A/B numbers are in DESIGN
// §5; the losing forms were removed in round 4):
//  * kPreFill ring items are issued in front of the x-tile wait, the rest after the transform: fewer
//    weight lines compete with the x tile's (cfg2 step -0.25 us against the whole fill in front, 0 in
//    front -0.1; profiles/r03g/prologue_ab.txt);
//  * the start point of a row is one 8-B load (elements 0..3), not 16 B (-0.08 us);
//  * small latent (SZ): only wave 0 (whose lanes hold mu, logvar) draws eps, in the prologue while
//    the x tile is in flight (C0 ‖ E0 2.44 -> 1.80 us, profiles/r03g/eps_ab.txt);
//  * wide latent: kEpsProWide of each wave's eps draws move from the E0 GEMM to the prologue — 1 of
//    4 in the e4m3 form (its E0 streams half the bytes; round 3 measured 2 against 0: step 54.8 ->
//    54.2 us; round 6 on the current chain 1 against 0 / 2 / 3 / 4: 46.72-46.74 us against
//    46.83-46.96 / 46.92-47.33 / 46.96-47.13 / 47.13-47.15, profiles/r06w/ab_epspro_*.json), none
//    in bf16 (its E0 is stream-bound; the prologue only grows: +0.3-0.9 us;
//    profiles/r03i/epswide_ab_*.txt);
//  * an L2 warm-up of E0's fragments in the prologue measured +0.7-1.0 us (profiles/r03g/warm_ab.txt)
//    and is not built.
#ifndef CVAE_WIDE_PREFILL
#define CVAE_WIDE_PREFILL 4  // diagnostic builds: A/B of the ring items issued before the x-tile wait
#endif
constexpr int kPreFill = CVAE_WIDE_PREFILL;
#ifndef CVAE_DIAG_EPS_PRO_F8
#define CVAE_DIAG_EPS_PRO_F8 1  // diagnostic builds only: the e4m3 form's prologue draws (A/B)
#endif
template <class A>
constexpr int kEpsProWide = A::F8 ? CVAE_DIAG_EPS_PRO_F8 : 0;
// one 16-B piece of fragment item at byte offset `off` from the arena base: a buffer load — lane·16
// is a loop-invariant voffset, the item's offset a scalar soffset (2-3 SALU per item); the 64-bit
// global address cost 3 VALU (one a 64-bit shift-add) + ~7 SALU per item (cfg2 step 26.6 -> 26.0
// us, profiles/r03g).  The e4m3 form needs the pad below (f8_pad): rounds 3-4 found its buffer-load
// build not repeatable and kept global loads with a scalar base (CVAE_F8_BUFLOAD=0; chain 41.4 ->
// 40.5 us then, profiles/r03g/saddr_ab.txt) — round 5 found the cause
// The e4m3 form's fragments are buffer loads too, with CVAE_F8_MFMA_PAD wait states between each
// e4m3 MFMA and the refill load that reuses its B operand's ring registers (round 5).  Without the pad
// the buffer-load build is not repeatable: 300 of 300 forward_backward calls differ
// (scripts/repeat_check.py, profiles/r05i/) — the refill's data lands in registers an e4m3 MFMA
// queued behind its predecessors has not read yet, a hazard hipcc does not pad for these
// instructions; with 16 states 0 of 300 differ.  The scalar-base global-load form (CVAE_F8_BUFLOAD=0)
// spends ~8 SALU and a 64-bit VALU add on each item's address, which happened to cover the hazard
// (0 of 300); buffer loads + pad run the chain 0.2 us faster.
#ifndef CVAE_F8_BUFLOAD
#define CVAE_F8_BUFLOAD 1
#endif
#ifndef CVAE_F8_MFMA_PAD
#define CVAE_F8_MFMA_PAD 16
#endif
// CVAE_F8_MFMA_PAD wait states after an e4m3 MFMA, before the refill load that reuses its operand registers
__device__ __forceinline__ void f8_pad() {
  if constexpr (CVAE_F8_MFMA_PAD > 0) {
    asm volatile("s_nop %0" ::"n"(CVAE_F8_MFMA_PAD > 8 ? 7 : CVAE_F8_MFMA_PAD - 1));
    if constexpr (CVAE_F8_MFMA_PAD > 8) asm volatile("s_nop %0" ::"n"(CVAE_F8_MFMA_PAD - 9));
  }
}
template <bool F8>
__device__ __forceinline__ bf16x8 wload(const char* AR, int64_t off, int lane) {
  if constexpr (!F8 || CVAE_F8_BUFLOAD) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)AR, (short)0, 0x7fffffff, 0x00020000);
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (int)off, 0));
  } else {  // global_load with a scalar base + a 32-bit lane offset
    typedef const __attribute__((address_space(1))) char* gchar;
    gchar p = (gchar)(AR + off);
    asm volatile("" : "+s"(p));
    return *(const __attribute__((address_space(1))) bf16x8*)(p + (uint32_t)(lane * 16));
  }
}

// stream item G of this wave → ring slot G % P (no-op past the end of the stream)
template <class A, int P, int G>
__device__ __forceinline__ void ring_load(Ring<P>& ring, const char* AR, int wave, int lane) {
  using PL = Plan<A>;
  if constexpr (G < PL::total) {
    constexpr int s = PL::step_of(G);
    constexpr StepInfo st = PL::step(s);
    constexpr int j = G - PL::start(s);
    constexpr int NGR = st.GRP ? st.TS / st.GRP : 1, GS = st.GRP ? st.GRP : st.TS;  // groups, slots per group
    constexpr int grp = j / (st.KC * GS), kc = (j / GS) % st.KC, slot = grp + NGR * (j % GS);
    constexpr int64_t base = st.bwd ? (st.F8 ? A::wb8(st.layer) : A::wb(st.layer)) : A::wf(st.layer);
    int w = wave;
    asm volatile("" : "+s"(w));  // recomputed per item: hoisted, ~400 item addresses would be live SGPRs
    int t = w + NW * slot;
    if constexpr (NW * (slot + 1) > st.NTL) t = min(t, st.NTL - 1);
    const int64_t frag = st.KS ? w + NW * kc : t * st.KC + kc;  // KS: tile 0, chunk = wave + 8·item
    if constexpr (st.KS && NW * (kc + 1) > A::FC_KCH) {
      // a K chunk past the layer (wave-uniform): no load, and gemm skips its MFMA
      if (w + NW * kc < A::FC_KCH) ring.r[G % P] = wload<A::F8>(AR, base + frag * 1024, lane);
    } else if constexpr (!st.KS && NW * (slot + 1) > st.NTL) {
      // a slot past the layer's tiles: no load (wave-uniform); the stale ring register feeds an
      // MFMA whose result the epilogue drops
      if (w + NW * slot < st.NTL) ring.r[G % P] = wload<A::F8>(AR, base + frag * 1024, lane);
    } else {
      ring.r[G % P] = CVAE_DIAG_NOWLOAD ? bf16x8{} : wload<A::F8>(AR, base + frag * 1024, lane);
    }
  }
}

// e4m3 activation images (F8): fragment order, 16 B per (64-wide K pair kp, row quad q, row r) —
// lane (r, q) of an e4m3 X operand reads its two 32-wide chunks of pair kp (frag_k order, as the
// e4m3 weight fragment, cvae_device.h f8_wf_off) with one ds_read_b128
__device__ __forceinline__ l2 x8frag(const void* img8, int kp) {
  const int lane = threadIdx.x & 63;
  return *(const l2*)((const uint8_t*)img8 + (((kp * 4 + (lane >> 4)) * 16 + (lane & 15)) << 4));
}
// rows 4q..4q+3 of feature f (f & 3 == lane & 3: a quad of lanes holds 4 consecutive features):
// e4m3 of the bf16 activation (RNE, saturated at ±448 as f8x8).  The quad's 4 x 4 block is
// transposed so lane b writes row 4q + b's 4 features as one dword; byte stores of single features
// were 16-way bank conflicts (the x_rel image cost 3.8 us of prologue that way).  The transpose is
// of the converted bytes (round 5): each lane packs its feature's 4 rows into one dword, takes the
// quad's four dwords by DPP broadcasts and gathers byte b of each with v_perm (≈17 VALU; transposing
// the fp32 values first, quad_t, cost ≈30)
__device__ __forceinline__ void img8(void* im8, int f, bf16x4 h, int q) {
  const int b = threadIdx.x & 3, f0 = f - b;
  const int kc = f0 >> 5, kk = f0 & 31, qx = (kk & 15) >> 2, e0 = (kk >> 4) << 2;
  // feature f, rows 4q..4q+3: fp32 from the two packed dwords (left to itself the compiler re-rounds
  // each value from fp32 instead, two more VALU per value)
  u32x2 hw = __builtin_bit_cast(u32x2, h);
  asm volatile("" : "+v"(hw));
  const f32x4 v = {__builtin_bit_cast(float, hw[0] << 16), __builtin_bit_cast(float, hw[0] & 0xffff0000u),
                   __builtin_bit_cast(float, hw[1] << 16), __builtin_bit_cast(float, hw[1] & 0xffff0000u)};
  auto c = [](float x) { return f8_sat(x); };
  int m = __builtin_amdgcn_cvt_pk_fp8_f32(c(v[0]), c(v[1]), 0, false);
  m = __builtin_amdgcn_cvt_pk_fp8_f32(c(v[2]), c(v[3]), m, true);  // byte i: row 4q + i
  const unsigned d0 = __builtin_amdgcn_update_dpp(0, m, 0x00, 0xF, 0xF, false),
                 d1 = __builtin_amdgcn_update_dpp(0, m, 0x55, 0xF, 0xF, false),
                 d2 = __builtin_amdgcn_update_dpp(0, m, 0xAA, 0xF, 0xF, false),
                 d3 = __builtin_amdgcn_update_dpp(0, m, 0xFF, 0xF, 0xF, false);
  const unsigned sel = (unsigned)b | ((unsigned)(b + 4) << 8);  // byte b of src1, byte b of src0
  const unsigned lo = __builtin_amdgcn_perm(d1, d0, sel), hi = __builtin_amdgcn_perm(d3, d2, sel);
  const int w = (int)__builtin_amdgcn_perm(hi, lo, 0x05040100u);  // byte j: feature f0 + j, row 4q + b
  *(int*)((uint8_t*)im8 + ((((kc >> 1) * 4 + qx) * 16 + 4 * q + b) << 4) + (kc & 1) * 8 + e0) = w;
}

// acc[slot] = X·Wᵀ for this wave's n-tiles of step S: X chunk kc read once (two transposed LDS
// reads; an e4m3 step: one read of the pair's e4m3 image), multiplied by every slot's fragment;
// each consumed ring slot is refilled P items ahead.  e4m3 steps: acc · sc (= 1/s) at the end.
template <bool F8>
using XOp = std::conditional_t<F8, l2, bf16x8>;
template <bool F8>
__device__ __forceinline__ XOp<F8> xop(const void* img, int kc) {
  if constexpr (F8) return x8frag(img, kc);
  else return xfrag((const __bf16*)img, kc);
}
template <bool F8>
__device__ __forceinline__ f32x4 xmfma(XOp<F8> x, bf16x8 w, f32x4 acc) {
  if constexpr (F8) {
    const l2 w8 = __builtin_bit_cast(l2, w);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(x[0], w8[0], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(x[1], w8[1], acc, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, w, acc, 0, 0, 0);
  }
}
// Two consecutive e4m3 K pairs in one block-scaled MFMA (16x16x128, unit E8M0 scales: 2x the
// rate of the non-scaled fp8 form, which runs at the bf16 rate on gfx950).  A lane's 32 bytes
// are its 16-B fragments of pairs kp and kp + 1, for A (activations) and B (weights) alike;
// scripts/ubench/mxcheck.hip checks this equals four v_mfma_f32_16x16x32_fp8_fp8 on the GPU.
template <class X>  // X = l2 (an e4m3 pair); the bf16 instantiation of the callers never reaches it
__device__ __forceinline__ f32x4 mx2(X x0, X x1, bf16x8 w0, bf16x8 w1, f32x4 acc) {
  static_assert(std::is_same<X, l2>::value, "e4m3 pairs only");
  const l2 w0l = __builtin_bit_cast(l2, w0), w1l = __builtin_bit_cast(l2, w1);
  typedef long l4 __attribute__((ext_vector_type(4)));
  const i32x8 a = __builtin_bit_cast(i32x8, l4{x0[0], x0[1], x1[0], x1[1]});
  const i32x8 b = __builtin_bit_cast(i32x8, l4{w0l[0], w0l[1], w1l[0], w1l[1]});
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
}
struct NoSide {
  template <class C>
  __device__ void operator()(C) const {}
};
// side(integral_constant<c>) runs after chunk c: VALU work placed inside a stream-bound GEMM
template <class A, int P, int S, int TS, class Side = NoSide>
__device__ __forceinline__ void gemm(Ring<P>& ring, const void* img, f32x4 (&acc)[TS], const char* AR, int wave,
                                     int lane, Side&& side = Side{}, float sc = 1.f) {
  using PL = Plan<A>;
  constexpr StepInfo st = PL::step(S);
  constexpr bool F8 = st.F8;
  static_assert(st.TS == TS && st.GRP == 0 && st.F8 != 2, "accumulator slots");
  constexpr int G0 = PL::start(S);
  sfor<0, TS>([&](auto t) { acc[decltype(t)::value] = f32x4{0.f, 0.f, 0.f, 0.f}; });
  static_assert(!st.KS || (TS == 1 && !F8), "K split: chunks wave, wave + 8, .. of one n-tile");
  if constexpr (st.KS) {  // chunk wave + 8c of the one n-tile; chunks past FC_KCH (wave-uniform) skipped
    sfor<0, st.KC>([&](auto kc) {
      constexpr int c = decltype(kc)::value, g = G0 + c;
      const int ch = wave + NW * c;
      if (NW * (c + 1) <= A::FC_KCH || ch < A::FC_KCH) {
        acc[0] = xmfma<false>(xop<false>(img, ch), ring.r[g % P], acc[0]);
        asm volatile("" : "+v"(acc[0]));
      }
      ring_load<A, P, g + P>(ring, AR, wave, lane);
      side(kc);
    });
    return;
  }
  XOp<F8> xf = xop<F8>(img, 0);
  XOp<F8> xe = xf;  // F8: the even pair, multiplied together with the odd one after it
  sfor<0, st.KC>([&](auto kc) {
    constexpr int c = decltype(kc)::value;
    // the next chunk's X fragment is read one chunk ahead
    const XOp<F8> xn = c + 1 < st.KC ? xop<F8>(img, c + 1) : xf;
    if constexpr (F8 && c % 2 == 0 && c + 1 < st.KC) {
      xe = xf;  // its MFMA (and refill) comes with pair c + 1
    } else if constexpr (F8 && c % 2 == 1) {
      sfor<0, TS>([&](auto t) {
        constexpr int u = decltype(t)::value, g0 = G0 + (c - 1) * TS + u, g = G0 + c * TS + u;
        acc[u] = mx2(xe, xf, ring.r[g0 % P], ring.r[g % P], acc[u]);
        asm volatile("" : "+v"(acc[u]));  // MFMA before the refills, as below
        f8_pad();
        ring_load<A, P, g0 + P>(ring, AR, wave, lane);
        ring_load<A, P, g + P>(ring, AR, wave, lane);
      });
    } else sfor<0, TS>([&](auto t) {
      constexpr int u = decltype(t)::value, g = G0 + c * TS + u;
      acc[u] = xmfma<F8>(xf, ring.r[g % P], acc[u]);
      // Program order MFMA(g) → refill(g + P): the empty volatile asm on the result is ordered
      // before the (volatile) address step of the refill.  Left alone, the scheduler issues a
      // step's refills first and sinks its MFMA chains, and every ring slot then needs a second
      // register (spills).
      asm volatile("" : "+v"(acc[u]));
      if constexpr (F8) f8_pad();
      ring_load<A, P, g + P>(ring, AR, wave, lane);
    });
    side(kc);
    xf = xn;
  });
  if constexpr (F8) sfor<0, TS>([&](auto t) { acc[decltype(t)::value] *= sc; });
}

// The grouped form (StepInfo::GRP > 0): all KC X chunks read first, then per group p its GRP
// accumulators over the whole K and epi(integral_constant<p>, acc) — the group's epilogue issues
// while the next group's fragments stream in.
template <class A, int P, int S, class Epi>
__device__ __forceinline__ void gemm_grouped(Ring<P>& ring, const void* img, const char* AR, int wave, int lane,
                                             Epi&& epi, float sc = 1.f) {
  using PL = Plan<A>;
  constexpr StepInfo st = PL::step(S);
  constexpr bool F8 = st.F8;
  static_assert(st.GRP > 0 && st.TS % st.GRP == 0, "grouped step");
  constexpr int G0 = PL::start(S), GS = st.GRP, NGR = st.TS / st.GRP, KC = st.KC;
  XOp<F8> xf[KC];
  sfor<0, KC>([&](auto kc) { xf[decltype(kc)::value] = xop<F8>(img, decltype(kc)::value); });
  sfor<0, NGR>([&](auto pp) {
    constexpr int p = decltype(pp)::value;
    f32x4 acc[GS];
    sfor<0, GS>([&](auto i) { acc[decltype(i)::value] = f32x4{0.f, 0.f, 0.f, 0.f}; });
    sfor<0, KC>([&](auto kc) {
      constexpr int c = decltype(kc)::value;
      if constexpr (F8 && c % 2 == 0 && c + 1 < KC) return;  // with pair c + 1 (mx2)
      if constexpr (F8 && c % 2 == 1) {
        sfor<0, GS>([&](auto i) {
          constexpr int u = decltype(i)::value, g0 = G0 + (p * KC + c - 1) * GS + u, g = G0 + (p * KC + c) * GS + u;
          acc[u] = mx2(xf[c - 1], xf[c], ring.r[g0 % P], ring.r[g % P], acc[u]);
          asm volatile("" : "+v"(acc[u]));
          f8_pad();
          ring_load<A, P, g0 + P>(ring, AR, wave, lane);
          ring_load<A, P, g + P>(ring, AR, wave, lane);
        });
        return;
      }
      sfor<0, GS>([&](auto i) {
        constexpr int u = decltype(i)::value, g = G0 + (p * KC + c) * GS + u;
        acc[u] = xmfma<F8>(xf[c], ring.r[g % P], acc[u]);
        asm volatile("" : "+v"(acc[u]));  // MFMA(g) before refill(g + P), as in gemm
        ring_load<A, P, g + P>(ring, AR, wave, lane);
      });
    });
    if constexpr (F8) sfor<0, GS>([&](auto i) { acc[decltype(i)::value] *= sc; });
    epi(pp, acc);
  });
}

// The e4m3 dX GEMM of an f8b layer (StepInfo::F8 == 2; BASELINE cfg5's last decoder layer, decoder
// L0 and fc): acc[slot] = G·W over the bf16 gradient image G, W streamed as e4m3(s·Wᵀ) K-pair
// fragments (Wb8), every two K pairs in one block-scaled MFMA.  MX blocks of the instruction
// (mapped on the GPU by scripts/ubench/mxscale.hip): lane r + 16j holds byte quarters h = 0..3 of
// row r; block b = 2·(h >> 1) + (j >> 1) — the 16-B half h >> 1 of the lane pair j >> 1 — and its
// E8M0 byte comes from lane r + 16b.  Quarter h of a lane here is its 8 values of gradient chunk
// 4g + h, so a block is 16 positions of each of two adjacent chunks of one row (oracle mx_dx).
// The operand is converted once per workgroup into LDS (mx_convert, a barrier, then gemm_mxb):
// each lane takes the exponents of its two halves' maxima, one permlane16 swap with its pair
// partner (lane ^ 16) makes them the block maxima, k = 134 − biased exponent = 7 − floor(log2
// max|G|) puts a block's largest value in [128, 256) (no saturation, no step state), and each half
// converts with its block's 2^k; in the GEMM lane j reads the exponent of block j (stored by the
// lanes of pair j & 1 of its row) for the scale operand.  B takes 1/s: the accumulator is the
// unscaled product.  The gradient rows span ~10^4 in magnitude (the start /
// time terms of dL/drecon beside the mean-squared ones), which one scale per tensor cannot hold.
__device__ __forceinline__ f32x4 mx2s(l2 x0, l2 x1, bf16x8 w0, bf16x8 w1, f32x4 acc, int sa, int sb) {
  const l2 w0l = __builtin_bit_cast(l2, w0), w1l = __builtin_bit_cast(l2, w1);
  typedef long l4 __attribute__((ext_vector_type(4)));
  const i32x8 a = __builtin_bit_cast(i32x8, l4{x0[0], x0[1], x1[0], x1[1]});
  const i32x8 b = __builtin_bit_cast(i32x8, l4{w0l[0], w0l[1], w1l[0], w1l[1]});
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa, 0, sb);
}
// The MX operand image of step S: wave w converts K-pair groups w, w + 8, .. of the bf16 gradient
// image (its four chunk fragments, mx_block) into e4m3 operand halves at twin + g·2 KB + h·1 KB +
// lane·16 and the lane pair's two block exponents at twin + NG·2 KB + (g·64 + lane)·4 — each group
// converted once per workgroup instead of by all 8 waves.  Both rounds' fragments are read before
// either converts.  The caller joins a barrier before gemm_mxb reads it.
template <class A, int S>
__device__ __forceinline__ void mx_convert(const __bf16* img, char* twin, int wave, int lane) {
  constexpr StepInfo st = Plan<A>::step(S);
  constexpr int KP = st.KC, NG = (KP + 1) / 2, NR = (NG + NW - 1) / NW;
  bf16x8 c[NR][4];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int g = r * NW + wave;
    if (NG % NW != 0 && g >= NG) break;  // wave-uniform
    const bool two = 2 * g + 1 < KP;      // an odd last pair: the second half of the block is zero
    c[r][0] = xfrag(img, 4 * g);
    c[r][1] = xfrag(img, 4 * g + 1);
    c[r][2] = two ? xfrag(img, 4 * g + 2) : bf16x8{};
    c[r][3] = two ? xfrag(img, 4 * g + 3) : bf16x8{};
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int g = r * NW + wave;
    if (NG % NW != 0 && g >= NG) break;
    l2 x0, x1;
    const unsigned e = mx_block(c[r], x0, x1);
    *(l2*)(twin + g * 2048 + lane * 16) = x0;
    *(l2*)(twin + g * 2048 + 1024 + lane * 16) = x1;
    *(unsigned*)(twin + NG * 2048 + (g * 64 + lane) * 4) = e;
  }
}
template <class A, int S>
constexpr int mx_twin_bytes() {
  constexpr int NG = (Plan<A>::step(S).KC + 1) / 2;
  return NG * (2048 + 256);
}
template <class A, int P, int S, int TS>
__device__ __forceinline__ void gemm_mxb(Ring<P>& ring, const char* twin, f32x4 (&acc)[TS], const char* AR, int wave,
                                         int lane, int sb) {
  using PL = Plan<A>;
  constexpr StepInfo st = PL::step(S);
  static_assert(st.F8 == 2 && st.TS == TS && st.GRP == 0 && !st.KS, "an MX dX step");
  constexpr int G0 = PL::start(S), KP = st.KC, NG = (KP + 1) / 2;  // K pairs (two 32-wide chunks each)
  sfor<0, TS>([&](auto t) { acc[decltype(t)::value] = f32x4{0.f, 0.f, 0.f, 0.f}; });
  sfor<0, NG>([&](auto gg) {
    constexpr int g = decltype(gg)::value, p0 = 2 * g, p1 = 2 * g + 1;
    constexpr bool two = p1 < KP;
    const l2 x0 = *(const l2*)(twin + g * 2048 + lane * 16), x1 = *(const l2*)(twin + g * 2048 + 1024 + lane * 16);
    // the scale this lane hands the instruction: block j = lane / 16 = (half j >> 1, lane pair j & 1),
    // whose exponent the lanes of pair j & 1 of this row stored
    const int j = lane >> 4;
    const unsigned ep = *(const unsigned*)(twin + NG * 2048 + (g * 64 + (lane & 15) + 32 * (j & 1)) * 4);
    const int sa = 127 - mx_k((int)(ep >> (16 * (j >> 1))) & 0xffff);
    sfor<0, TS>([&](auto t) {
      constexpr int u = decltype(t)::value, ga = G0 + p0 * TS + u, gb = G0 + (two ? p1 : p0) * TS + u;
      acc[u] = mx2s(x0, x1, ring.r[ga % P], ring.r[gb % P], acc[u], sa, sb);
      asm volatile("" : "+v"(acc[u]));  // MFMA before the refills (as gemm)
      f8_pad();
      ring_load<A, P, ga + P>(ring, AR, wave, lane);
      if constexpr (two) ring_load<A, P, gb + P>(ring, AR, wave, lane);
    });
  });
}

// the first P items of the stream (prologue)
template <class A, int P>
__device__ __forceinline__ void ring_fill(Ring<P>& ring, const char* AR, int wave, int lane) {
  sfor<0, P>([&](auto g) { ring_load<A, P, decltype(g)::value>(ring, AR, wave, lane); });
}

// Arena stores.  An epilogue only writes LDS; the arena copy of each LDS image (the layer's
// feature-major [Kf][16 rows] slab of this row tile, exactly the image's content) is issued in the
// NEXT step, while the image is still intact, as 16-B stores: per-CU store ISSUE bounds these
// (MI355X_MICROARCH.md, store tail: 16-B stores halve it against the 8-B-per-lane epilogue
// stores of a lane's 4 rows), and they leave the epilogue's critical path.  Write-through (sc1):
// the lines leave L2 now, for the dW kernel behind, not at the kernel-end writeback.
// The arena as a buffer resource: the 16-B stores are buffer_store_dwordx4 with the sc1 cache
// policy (aux 16 on gfx950) through the builtin, so the compiler sees their operands.  (They were
// an inline-asm global_store: with a one-lane f64 block added to the prologue, the stores of a
// few lanes then wrote stale data — the hazard recognizer cannot see into inline asm.)
struct ArenaDst {
  __amdgpu_buffer_rsrc_t rs;
  const char* base;
};
__device__ __forceinline__ ArenaDst arena_dst(const char* AR) {
  return ArenaDst{__builtin_amdgcn_make_buffer_rsrc((void*)AR, (short)0, 0x7fffffff, 0x00020000), AR};
}
__device__ __forceinline__ void st16(const ArenaDst& d, const void* p, u32x4 v) {
  if (CVAE_DIAG_NOSTORE) return;
  __builtin_amdgcn_raw_buffer_store_b128(v, d.rs, (int)((const char*)p - d.base), 0, 16);  // sc1
}

// rounds [R0, R1) of the 16-B copy of features [0, NF) of an LDS image (ioff layout) to the arena
// matrix `mat` (Kf feature rows) at feature offset goff: task k = feature k / 2, rows 8(k & 1)..+7.
// In the image, row quad q of feature f sits at slot q ^ x (x = (f >> 2) & 3), so a task's two
// quads are the slot pair 2(h ^ (x >> 1)), +1, in swapped order when x is odd.
// Threads T0.. take the tasks (T0 = 256: a 128-feature image on waves 4-7, beside another on 0-3).
template <int NF, int R0, int R1, int T0 = 0>
__device__ __forceinline__ void img_copy(const __bf16* img, const ArenaDst& dst, void* mat, int Kf, int goff, int b0) {
#pragma unroll
  for (int r = R0; r < R1; ++r) {
    if (r * NT - T0 >= 2 * NF) break;
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));  // per-round addresses: hoisted, every round's would stay live
    const int k = r * NT + t - T0;
    if ((T0 == 0 && 2 * NF % NT == 0) || (k >= 0 && k < 2 * NF)) {
      const int f = k >> 1, h = k & 1, x = (f >> 2) & 3;
      u32x4 v = *(const u32x4*)(img + f * 16 + 8 * (h ^ (x >> 1)));
      if (x & 1) v = u32x4{v[2], v[3], v[0], v[1]};
      st16(dst, (__bf16*)mat + aoff(goff + f, b0 + 8 * h, Kf), v);
    }
  }
}

// TAP (parity tests only, cvae_tap_outputs): the chain also writes what its epilogues computed —
// recon (the last decoder layer's output before the loss, fp32 (batch, S, D)), mu and logvar (fp32
// (batch, Z)) — to a.recon_out / a.mu_out / a.lv_out: the training step's own rounding points
// XB: bf16 rows only (the bench's and the peer step's data) — the fp32-row load path compiled out.
// Both row formats behind a runtime branch share the x registers, and the compiler's merged wait
// counts then hold the first Philox draw until the whole x tile has landed; fp32 rows keep the
// runtime form (a compile-time fp32 form needs 142 VGPRs: tests/test_kernel_resources.py)
template <class A, int P, bool TAP = false, bool XB = false>
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
  // F8 only: the e4m3 twins of the bf16 images that feed e4m3 GEMMs (A::twin_off), and 1/s per layer
  float* const INVS = (float*)(smem + A::L_INVS);
  // the X operand of step S from the bf16 image at LDS offset L: its e4m3 twin for an e4m3 GEMM
  auto opnd = [smem](auto sI, auto LI) -> const void* {
    constexpr int L = decltype(LI)::value;
    if constexpr (PL::step(decltype(sI)::value).F8) return smem + A::twin_off(L);
    else return smem + L;
  };
  auto scl = [INVS](auto sI) -> float {
    if constexpr (PL::step(decltype(sI)::value).F8) return INVS[PL::step(decltype(sI)::value).layer];
    else return 1.f;
  };
  // diagnostic builds only: thread 0's time at every step barrier, kept in LDS, written at the end
  unsigned long long* const STAMPS = (unsigned long long*)(smem + A::L_STAMPS);
  int stamp_i = 0;
  auto bar = [&]() {
    lbar();
    if (CVAE_DIAG_STAMPS && threadIdx.x == 0 && stamp_i < 64) STAMPS[stamp_i] = __builtin_amdgcn_s_memrealtime();
    ++stamp_i;
  };
  if (CVAE_DIAG_STAMPS && threadIdx.x == 0) STAMPS[stamp_i++] = __builtin_amdgcn_s_memrealtime();
  // a stamp inside a step (CVAE_DIAG_STAMPS == 2 only)
  auto sub = [&]() {
    if (CVAE_DIAG_STAMPS == 2 && threadIdx.x == 0 && stamp_i < 64) STAMPS[stamp_i] = __builtin_amdgcn_s_memrealtime();
    if (CVAE_DIAG_STAMPS == 2) ++stamp_i;
  };
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
  const ArenaDst dst = arena_dst(AR);
  const int n = 16 * wave + n16;  // this lane's feature in the 128-wide layers (n-tile = wave)
  auto img = [&](__bf16* im, int f, bf16x4 v) { *(bf16x4*)(im + ioff(f, q)) = v; };
  // an image (LDS offset L) that feeds an e4m3 GEMM (F8): the bf16 image (the arena copy) and its
  // e4m3 twin
  auto img2 = [smem, q](auto LI, int f, bf16x4 v) {
    constexpr int L = decltype(LI)::value;
    *(bf16x4*)((__bf16*)(smem + L) + ioff(f, q)) = v;
    if constexpr (A::F8) img8(smem + A::twin_off(L), f, v, q);
  };
  using std::integral_constant;
  using IA0 = integral_constant<int, A::L_A0>;
  using IA1 = integral_constant<int, A::L_A1>;
  using ICB = integral_constant<int, A::L_CB>;
  using IHC = integral_constant<int, A::L_HCAT>;
  using IDC = integral_constant<int, A::L_DCAT>;

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
  using std::integral_constant;

  // the Philox offset of this launch: a scalar load before anything else (a vector load here, under
  // the counter-pointer branch, made the compiler drain every in-flight load at the fc step)
  const uint64_t rng_off = a.ctr ? *(const __attribute__((address_space(4))) uint64_t*)a.ctr : a.offset;

  Ring<P> ring;
  // a dX GEMM of step S over the bf16 gradient image: e4m3 with MX scales where the layer is f8b
  // MX operand images: the last decoder layer's in the recon time-channel buffers (dead after the
  // fix-up step), decoder L0's and fc's in the x_rel / dL/drecon image (dead once its arena copy is out)
  auto dgemm = [&](auto sI, const __bf16* gimg, auto& acc) {
    constexpr int S_ = decltype(sI)::value;
    constexpr StepInfo st = PL::step(S_);
    constexpr int TS_ = st.TS;
    if constexpr (st.F8 == 2) {  // B's E8M0 scale: the exponent byte of 1/s (a power of two)
      constexpr int TW = st.layer == A::LDL ? A::L_RCH0 : A::L_XIN;
      static_assert(st.layer == A::LDL ? mx_twin_bytes<A, S_>() <= 2 * S * R * 4
                                       : (mx_twin_bytes<A, S_>() <= Ip * 32 && S_ > PL::sDLb),
                    "MX operand image");
      mx_convert<A, S_>(gimg, smem + TW, wave, lane);
      lbar();
      sub();
      gemm_mxb<A, P, S_, TS_>(ring, smem + TW, acc, AR, wave, lane, (int)((__float_as_uint(INVS[st.layer]) >> 23) & 0xff));
    } else
      gemm<A, P, S_, TS_>(ring, gimg, acc, AR, wave, lane);
  };
  constexpr int PF0 = kPreFill < P ? kPreFill : P;  // ring items issued before the x-tile wait
  float s_recon = 0.f, s_kl = 0.f, s_start = 0.f, s_t0 = 0.f, s_relu = 0.f;

  // eps of the reparameterisation (:199-206), per mu tile k of this lane (latent j, rows 4q..4q+3):
  // host-given (loaded unconditionally — rows clamped into the batch, any valid address when eps
  // is drawn in-kernel — a load under a branch drains the weight stream) or Philox keyed by the
  // global row (data parallelism: eps_row0 = the rank's first row).  The Philox draws (integer
  // multiplies and transcendentals, ~0.3 us of VALU per wave) run inside the stream-bound
  // encoder-L1 GEMM, or (SZ) in the prologue while the x tile is in flight.
  // SZ: one tile of latents, held by wave 0's lanes n16 < Z (only wave 0 draws)
  constexpr int NZT = A::SZ ? 1 : Z / 128;
  f32x4 ep[NZT];
  const int rowq = 4 * q + (n16 & 3);  // the row this lane draws (4 latents) before the quad transpose
  auto eps_j0 = [&](int k) { return A::SZ ? min(4 * (n16 >> 2), Z - 4) : 16 * (wave + NW * k) + 4 * (n16 >> 2); };
  auto eps_load = [&](int k) {
    const int j0 = eps_j0(k);
    const float* const ebase = a.eps ? a.eps : (const float*)(AR + A::bias_base);  // global memory either way
    const int erow = a.eps ? min(b0 + rowq, max(a.batch - 1, 0)) : 0;
    return gld<f32x4>(ebase + (a.eps ? (size_t)erow * Z + j0 : 0));
  };
  auto eps_make = [&](auto kk, f32x4 eh) {
    constexpr int k = decltype(kk)::value;
    const int j0 = eps_j0(k);
    // the draw first and the host value picked last: with the pick first the compiler copied the
    // host-eps registers before the draw, and the draw waited for that load — in flight behind the
    // x tile — even when the kernel draws (the host-eps path draws for nothing: parity tests only)
    const f32x4 d = philox_normal4(a.seed, rng_off, (uint32_t)(a.eps_row0 + b0 + rowq), (uint32_t)j0);
    f32x4 e = a.eps ? eh : d;
    if (rowq >= nrows) e = f32x4{0.f, 0.f, 0.f, 0.f};
    ep[k] = quad_t(e);
  };
  auto draw_eps = [&](auto kk) { eps_make(kk, eps_load(decltype(kk)::value)); };
  constexpr bool EPS_PRO = A::SZ;  // the draw sits in the prologue
  // wide latent (NZT tiles per wave): draws 0 .. NPRO-1 in the prologue, the rest in the E0 GEMM
  constexpr int NPRO = EPS_PRO ? 1 : (kEpsProWide<A> < NZT ? kEpsProWide<A> : NZT);
  // SZ: the draw runs on the last wave — no x-transform task at cfg2's 200 tasks, and its SIMD's
  // other wave (3) has the lightest one — and reaches wave 0's lanes (which hold mu, logvar)
  // through LDS across the prologue barrier (the recon time-channel buffer, idle until the loss)
  const bool eps_mine = !A::SZ || wave == NW - 1;  // wave-uniform
  // SZ: the eps hand-off (last wave → wave 0) in the recon time-channel buffer — in an F8 layout that
  // offset is also the e4m3 input / decoder-input twin the prologue writes
  static_assert(!(A::SZ && A::F8), "EPSX would overlap L_X8 / L_DCAT8");
  float* const EPSX = (float*)(smem + A::L_RCH0);

  // ---- prologue: x tile (relative transform, Training_VAE.py:345-348), biases, LDS pads
  // x_f32 (CVAE_X_F32: real data with ~200 m absolute coordinates): fp32 rows, the start point
  // subtracted in fp32 and the relative offsets rounded to bf16 once
  {
    // Task = one timestep pair (12 features: 24 B of a bf16 row, 48 B of an fp32 row) of the four
    // rows of one row quad: the thread holds all 4 rows of every feature it writes, so the
    // feature-major image is a register transpose (v_perm / v_cvt_pk), with no DPP or selects; only
    // the features with d = 1, 2 are rebased, the rest of a bf16 row are copied bit for bit (x − 0
    // rounds to x).  Round 5: this was 719 VALU per wave for 16-B row vectors + quad transposes.
    static_assert(D == 6 && I % 12 == 0, "x_rel transform: 12-feature timestep pairs (D == 6)");
    constexpr int NKT = I / 12, NTASK = 4 * NKT;  // timestep pairs per row; tasks per tile
    static_assert(NTASK <= NT, "x_rel transform: one task per thread");
    const int last = max(a.batch - 1, 0);
    const bool x32 = !XB && a.x_f32 != 0;
    const int xt = min(tid, NTASK - 1), xrq = xt / NKT, xk = xt - xrq * NKT;  // idle threads: task NTASK-1, no store
    uint32_t xw[4][12];  // row 4xrq + i: dwords of its 12 features (bf16: [0..5])
    uint32_t xs[4][2];   // its start point x[:,0,1:3] (Training_VAE.py:345): bf16 dwords 0, 1 / fp32 features 1, 2
    // x tile loads, as four straight-line paths (with and without a row gather, fp32 or bf16 rows:
    // block-uniform branches outside the loads).  A gather load, or the x32 branch, inside the row
    // loop made the compiler wait for each row's x loads before the next row's (its wait counts
    // merge at every join, and the no-gather bf16 path paid for the others too) — four serial round
    // trips in the prologue
    auto x_loads = [&](auto gather, auto f32rows) {
      const uint32_t* pr[4];  // row starts, all before the first x load (a gather: one wait)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int64_t g = min(b0 + 4 * xrq + i, last);
        if constexpr (decltype(gather)::value) g = gld<int64_t>(a.idx + g);
        pr[i] = decltype(f32rows)::value ? (const uint32_t*)a.x + g * I
                                         : (const uint32_t*)((const __bf16*)a.x + g * I);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t* const p = pr[i];
        if constexpr (decltype(f32rows)::value) {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const u32x4 v = gld<u32x4>(p + 12 * xk + 4 * j);
#pragma unroll
            for (int e = 0; e < 4; ++e) xw[i][4 * j + e] = v[e];
          }
          xs[i][0] = gld<uint32_t>(p + 1);
          xs[i][1] = gld<uint32_t>(p + 2);
        } else {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const u32x2 v = gld<u32x2>(p + 6 * xk + 2 * j);
            xw[i][2 * j] = v[0];
            xw[i][2 * j + 1] = v[1];
          }
          const u32x2 v0 = gld<u32x2>(p);
          xs[i][0] = v0[0];
          xs[i][1] = v0[1];
        }
      }
    };
    if (a.idx) {
      if (x32) x_loads(std::true_type{}, std::true_type{});
      else x_loads(std::true_type{}, std::false_type{});
    } else {
      if (x32) x_loads(std::false_type{}, std::true_type{});
      else x_loads(std::false_type{}, std::false_type{});
    }
    // EPS_PRO: the host-eps load right behind the x tile (the x wait then covers it)
    f32x4 eh0[NPRO > 0 ? NPRO : 1];
    sfor<0, NPRO>([&](auto kk) { eh0[decltype(kk)::value] = eps_load(decltype(kk)::value); });
    constexpr int NB4 = A::nbias / 4, UB = (NB4 + NT - 1) / NT;
    f32x4 bv[UB];
#pragma unroll
    for (int k = 0; k < UB; ++k) bv[k] = gld<f32x4>((const float*)(AR + A::bias_base) + 4 * min(k * NT + tid, NB4 - 1));
    float invv = 1.f;  // F8: 1/s of layer tid (F8Scale::inv_s in front of its Wf)
    // wave 0 only (lanes < NL; wave-uniform branch): the selects cost ~50 VALU, on the prologue's
    // critical path in every wave that ran them
    if (A::F8 && wave == 0) {  // offsets selected from compile-time constants (a runtime A::wf(tid) is a loop)
      int64_t o = A::bias_base;
      sfor<0, A::NL>([&](auto ll) {
        constexpr int l = decltype(ll)::value;
        if constexpr (A::f8(l)) o = tid == l ? A::wf(l) - (int64_t)sizeof(F8Scale) + 4 : o;
      });
      invv = gld<float>((const float*)(AR + o));
    }
    // CLS: this tile's class ids (gathered like x) and the embedding table's operand copy (2 KB)
    int cid = -1;
    u32x4 tab = {0u, 0u, 0u, 0u};
    if constexpr (A::CLS) {
      if (tid < R) {
        int64_t g = min(b0 + tid, last);
        if (a.idx) g = gld<int64_t>(a.idx + g);
        const int c = a.classes ? gld<int>(a.classes + g) : 0;
        cid = tid < nrows ? min(max(c, 0), a.ncls - 1) : -1;  // out-of-range ids clamp (host validates)
      }
      if (tid < 2 * A::Np(A::LCE) * A::Kp(A::LCE) / 16) tab = gld<u32x4>(AR + A::wf(A::LCE) + 16 * tid);
    }
    // the weight stream queues behind the x tile and the biases (vmcnt retires in order)
    // the first PF0 items of the stream here, the rest after the x-tile transform (kPreFill)
    sfor<0, PF0>([&](auto g) { ring_load<A, P, decltype(g)::value>(ring, AR, wave, lane); });
    sfor<0, NPRO>([&](auto kk) {  // the Philox VALU issues while the x tile is in flight
      constexpr int k = decltype(kk)::value;
      if (CVAE_DIAG_NOPHILOX || !eps_mine) ep[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      else eps_make(kk, eh0[k]);
    });
    if constexpr (A::SZ)
      if (wave == NW - 1) *(f32x4*)(EPSX + 4 * lane) = ep[0];
    // device counters: this launch begins optimizer step ctr[1] + 1 and precomputes its Adam
    // scalars for the dW kernel behind it.  One wave of block 0, wave-uniformly, while it waits for
    // the x tile: the step count by scalar load, the f64 pow on every lane, one lane stores (at
    // the kernel's end, one lane's f64 pow delays the chain's completion).  Not the eps wave (SZ:
    // the last one) and, at cfg2's 200 transform tasks, a wave without one
    if (a.ctr && blk == 0 && wave == (A::SZ ? NW - 2 : NW - 1)) {
      const uint64_t t = *(const __attribute__((address_space(4))) uint64_t*)(a.ctr + 1) + 1;
      float s0 = 0.f, s1 = 0.f;
      if (a.adam_pre && !CVAE_DIAG_NOADAMPRE) adam_scalars(a.lr, a.beta1, a.beta2, (double)t, s0, s1);
      if (lane == 0) {  // agent-scope stores: the lines leave this CU's cache at once
        __hip_atomic_store(a.ctr + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.adam_pre)
          __hip_atomic_store(a.ctr + 2, __builtin_bit_cast(uint64_t, adam_f32x2{s0, s1}), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    sub();
    if (tid < 28 * 4) *(uint64_t*)(CIN + (4 + tid / 4) * 16 + 4 * (tid & 3)) = 0ull;
    if (tid < (Ip - I) * 4) *(uint64_t*)(XIN + (I + tid / 4) * 16 + 4 * (tid & 3)) = 0ull;
    if constexpr (A::Kp(A::LD0) > A::ZH)  // decoder-input K padding (read by D0, copied to xT(D0))
      if (tid < (A::Kp(A::LD0) - A::ZH) * 4) *(uint64_t*)(DCAT + (A::ZH + tid / 4) * 16 + 4 * (tid & 3)) = 0ull;
#pragma unroll
    for (int k = 0; k < UB; ++k)
      if (k * NT + tid < NB4) ((f32x4*)BIAS)[k * NT + tid] = bv[k];
    if constexpr (A::CLS) {
      if (tid < R) ((int*)(smem + A::L_CLSID))[tid] = cid;
      if (tid < 2 * A::Np(A::LCE) * A::Kp(A::LCE) / 16) ((u32x4*)(smem + A::L_CTAB))[tid] = tab;
    }
    if (A::F8 && wave == 0) {
      bool f8l = false;
      sfor<0, A::NL>([&](auto ll) { f8l = f8l || (A::f8(decltype(ll)::value) && tid == decltype(ll)::value); });
      if (tid < A::NL) INVS[tid] = f8l ? invv : 1.f;
    }
    if (nrows < R) {  // block-uniform: the batch's last tile; rows past it are zero
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool live = 4 * xrq + i < nrows;
#pragma unroll
        for (int e = 0; e < 12; ++e) xw[i][e] = live ? xw[i][e] : 0u;
        xs[i][0] = live ? xs[i][0] : 0u;
        xs[i][1] = live ? xs[i][1] : 0u;
      }
    }
    auto f32 = [](uint32_t u) { return __builtin_bit_cast(float, u); };
    auto pk = [](float lo, float hi) {  // two fp32 → bf16 (RNE), lo in bits 0..15
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      return __builtin_bit_cast(uint32_t, bf16x2{(__bf16)lo, (__bf16)hi});
    };
    float S0[4], S1[4];  // the rows' start point as fp32
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      S0[i] = x32 ? f32(xs[i][0]) : f32(xs[i][0] & 0xffff0000u);
      S1[i] = x32 ? f32(xs[i][1]) : f32(xs[i][1] << 16);
    }
    if (tid < NTASK) {
      char* const xb = (char*)XIN + 384 * xk;  // features 12xk .. 12xk+11, 32 B each (ioff)
      int sw[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) sw[c] = 8 * (xrq ^ ((3 * xk + c) & 3));
#pragma unroll
      for (int f = 0; f < 12; ++f) {
        const int d = f % D;
        u32x2 o;
        if (x32 || d == 1 || d == 2) {  // x32 is block-uniform
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float x = x32 ? f32(xw[i][f]) : f32((f & 1) ? (xw[i][f >> 1] & 0xffff0000u) : (xw[i][f >> 1] << 16));
            v[i] = d == 1 ? x - S0[i] : d == 2 ? x - S1[i] : x;
          }
          o = u32x2{pk(v[0], v[1]), pk(v[2], v[3])};
        } else {  // bf16, not rebased: the halves as they are
          const uint32_t sel = (f & 1) ? 0x07060302u : 0x05040100u;
          o = u32x2{__builtin_amdgcn_perm(xw[1][f >> 1], xw[0][f >> 1], sel),
                    __builtin_amdgcn_perm(xw[3][f >> 1], xw[2][f >> 1], sel)};
        }
        *(u32x2*)(xb + 32 * f + sw[f >> 2]) = o;
      }
      if (xk == 0) {  // the condition input (x, y, 0, 0) of the rows (c_start, :345): CIN features 0..3
        char* const cb = (char*)CIN + 8 * xrq;
        *(u32x2*)(cb) = u32x2{pk(S0[0], S0[1]), pk(S0[2], S0[3])};
        *(u32x2*)(cb + 32) = u32x2{pk(S1[0], S1[1]), pk(S1[2], S1[3])};
        *(u32x2*)(cb + 64) = u32x2{0u, 0u};
        *(u32x2*)(cb + 96) = u32x2{0u, 0u};
      }
    }
  }
  sfor<PF0, P>([&](auto g) { ring_load<A, P, decltype(g)::value>(ring, AR, wave, lane); });
  sub();
  bar();
  if constexpr (A::SZ)
    if (wave == 0) ep[0] = *(const f32x4*)(EPSX + 4 * lane);
  if constexpr (A::CLS) {
    // the one-hot class image (xT(LCE)) and e = table[class] into both concatenations at 2H + k and
    // Z + H + k (bf16: what one-hot · Wf(LCE) gives the generic chain; zeros in the K padding)
    const int* CLSID = (const int*)(smem + A::L_CLSID);
    const __bf16* TAB = (const __bf16*)(smem + A::L_CTAB);
    const int f = (tid >> 2) & 31, qq = tid & 3;
    bf16x4 v;
    if (tid < 128) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (__bf16)(CLSID[4 * qq + i] == f ? 1.f : 0.f);
      *(bf16x4*)((__bf16*)(smem + A::L_CLS1H) + ioff(f, qq)) = v;
    } else if (tid < 256) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = CLSID[4 * qq + i];
        v[i] = (c >= 0 && f < a.cdim) ? TAB[frag_off<__bf16>(f, c, A::Kp(A::LCE))] : (__bf16)0.f;
      }
      *(bf16x4*)((__bf16*)(smem + A::L_HCAT) + ioff(2 * H + f, qq)) = v;
      if (A::ZH + f < A::Kp(A::LD0)) *(bf16x4*)((__bf16*)(smem + A::L_DCAT) + ioff(A::ZH + f, qq)) = v;
    }
  }

  const float Bf = (float)a.batch;
  const float inv_BSD = 1.f / (Bf * (float)(S * D)), inv_2B = 1.f / (2.f * Bf), inv_B = 1.f / Bf;
  const float inv_BS1 = S > 1 ? 1.f / (Bf * (float)(S - 1)) : 0.f, inv_BZ = 1.f / (Bf * (float)Z);
  const bool use_start = a.w_start > 0.f, use_time = a.w_time > 0.f;  // Training_VAE.py:247, :256
  // the x_rel image → xT(E0): rounds of its 16-B copy, over the first encoder steps (done before
  // the loss epilogue overwrites XIN)
  constexpr int XR = (2 * Ip + NT - 1) / NT;
  static_assert(XR <= 5 && NE >= 4, "the x_rel copy runs over C0|E0, C1|E1, E2, E3");

  constexpr int ES = PL::step(PL::sE0).F8 ? 4 : 8;  // encoder-L1 K items between two draws
  auto eps_side = [&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if constexpr (c % ES == 2 && c / ES >= NPRO && c / ES < NZT) {
      if (CVAE_DIAG_NOPHILOX) ep[c / ES] = f32x4{0.f, 0.f, 0.f, 0.f};  // timing only
      else if (eps_mine) draw_eps(integral_constant<int, c / ES>{});
      else ep[c / ES] = f32x4{0.f, 0.f, 0.f, 0.f};  // SZ: only wave 0's lanes hold the latents
    }
  };
  static_assert(ES * (NZT - 1) + 2 < PL::step(PL::sE0).KC, "the eps draws fit in the encoder-L1 GEMM");

  // ================================================================ forward
  {  // C0 ‖ E0
    f32x4 acc[1];
    gemm<A, P, 0>(ring, CIN, acc, AR, wave, lane);
    img_copy<32, 0, 1>(CIN, dst, XT(A::LC0), A::Kp(A::LC0), 0, b0);
    img_copy<Ip, 0, 2>(XIN, dst, XT(A::LE0), A::Kp(A::LE0), 0, b0);
    img2(ICB{}, n, relu(acc[0], bias(A::LC0, n), integral_constant<int, A::MC0>{}));
    if constexpr (A::F8) {
      // the e4m3 twin of x_rel, one 64-wide K pair per wave at a time: lane (r, q) converts its own
      // MFMA fragment (two transposed bf16 reads, f8x8) — each pair once, not once per wave (as an
      // on-the-fly conversion inside the E0 GEMM: +2.6 us), and off the prologue (the unrolled
      // prologue form cost it 2 us); one extra barrier
      uint8_t* const X8 = (uint8_t*)(smem + A::L_X8);
#pragma nounroll
      for (int kp = wave; kp < A::NKI / 2; kp += NW)
        *(l2*)(X8 + (((kp * 4 + (lane >> 4)) * 16 + (lane & 15)) << 4)) =
            l2{f8x8(xfrag(XIN, 2 * kp)), f8x8(xfrag(XIN, 2 * kp + 1))};
      lbar();
    }
    sub();
    constexpr integral_constant<int, PL::sE0> sE0{};
    gemm<A, P, PL::sE0>(ring, opnd(sE0, integral_constant<int, A::L_XIN>{}), acc, AR, wave, lane, eps_side, scl(sE0));
    sub();
    img2(IA0{}, n, relu(acc[0], bias(A::LE0, n), integral_constant<int, A::ME(0)>{}));
  }
  bar();
  {  // C1 ‖ E1: h_c goes to both concatenations (fc input at H+n, decoder input at Z+n)
    f32x4 acc[1];
    constexpr integral_constant<int, PL::sC1> sC1{};
    gemm<A, P, PL::sC1>(ring, opnd(sC1, ICB{}), acc, AR, wave, lane, NoSide{}, scl(sC1));
    img_copy<H, 0, 1, 2 * H>(CB, dst, XT(A::LC1), H, 0, b0);
    img_copy<Ip, 2, 3>(XIN, dst, XT(A::LE0), A::Kp(A::LE0), 0, b0);
    const bf16x4 hc = relu(acc[0], bias(A::LC1, n), integral_constant<int, A::MC1>{});
    img2(IHC{}, H + n, hc);
    img2(IDC{}, Z + n, hc);
  }
  // encoder layers 1 .. NE-1 (input image: E(i-1)'s output, A0 for odd i); the last → h_traj
  sfor<1, NE>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    if constexpr (i > 1) bar();
    __bf16* const in = (i & 1) ? A0 : A1;
    f32x4 acc[1];
    constexpr integral_constant<int, PL::sC1 + i> sI{};
    using IIN = std::conditional_t<(i & 1), IA0, IA1>;
    using IOUT = std::conditional_t<i == NE - 1, IHC, std::conditional_t<(i & 1), IA1, IA0>>;
    gemm<A, P, PL::sC1 + i>(ring, opnd(sI, IIN{}), acc, AR, wave, lane, NoSide{}, scl(sI));
    img_copy<H, 0, 1>(in, dst, XT(A::LE(i)), H, 0, b0);
    if constexpr (i >= 2 && i <= 3) img_copy<Ip, i + 1, i + 2>(XIN, dst, XT(A::LE0), A::Kp(A::LE0), 0, b0);
    if constexpr (A::CLS && i == 1)
      img_copy<A::Kp(A::LCE), 0, 1, 2 * H>((const __bf16*)(smem + A::L_CLS1H), dst, XT(A::LCE), A::Kp(A::LCE), 0, b0);
    const bf16x4 he = relu(acc[0], bias(A::LE(i), n), integral_constant<int, A::ME(i)>{});
    img2(IOUT{}, n, he);
  });
  bar();
  // fc_mu ‖ fc_logvar (:195-196) + reparameterize (:199-206) + KL terms (:243): group k = the mu
  // tile wave + 8k and the logvar tile Z/16 + wave + 8k of the same latents
  f32x4 mu[NZT], lv[NZT];
  if constexpr (A::SZ) {  // one n-tile, K split over the waves; the partial sums meet in LDS
    float* const PFC = (float*)(smem + A::L_PFC);
    f32x4 acc[1];
    gemm<A, P, PL::sFC>(ring, HCAT, acc, AR, wave, lane);
    img_copy<A::Kp(A::LFC), 0, (2 * A::Kp(A::LFC) + NT - 1) / NT>(HCAT, dst, XT(A::LFC), A::Kp(A::LFC), 0, b0);
    *(f32x4*)(PFC + (wave * 16 + n16) * R + 4 * q) = acc[0];
    bar();
    if (wave == 0 && n16 < Z) {  // latent j = n16: mu at feature j, logvar at Z + j
      const int j = n16;
      f32x4 sm = {0.f, 0.f, 0.f, 0.f}, sl = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < NW; ++w) {  // fixed order: deterministic
        sm += *(const f32x4*)(PFC + (w * 16 + j) * R + 4 * q);
        sl += *(const f32x4*)(PFC + (w * 16 + Z + j) * R + 4 * q);
      }
      const float bm = bias(A::LFC, j), bl = bias(A::LFC, Z + j);
      f32x4 z;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        mu[0][i] = sm[i] + bm;
        lv[0][i] = sl[i] + bl;
        const float sd = __expf(0.5f * lv[0][i]);
        z[i] = mu[0][i] + ep[0][i] * sd;
        if (4 * q + i < nrows) s_kl += 1.f + lv[0][i] - mu[0][i] * mu[0][i] - __expf(lv[0][i]);
        if (TAP && 4 * q + i < nrows) {
          if (a.mu_out) a.mu_out[(size_t)(b0 + 4 * q + i) * Z + j] = mu[0][i];
          if (a.lv_out) a.lv_out[(size_t)(b0 + 4 * q + i) * Z + j] = lv[0][i];
        }
      }
      img(DCAT, j, to_bf4(z));
    }
  } else
  gemm_grouped<A, P, PL::sFC>(ring, opnd(integral_constant<int, PL::sFC>{}, IHC{}), AR, wave, lane, [&](auto kk, f32x4(&acc)[2]) {
    constexpr int k = decltype(kk)::value;
    if constexpr (k == 0) img_copy<2 * H, 0, 1>(HCAT, dst, XT(A::LFC), A::Kp(A::LFC), 0, b0);
    const int j = 16 * (wave + NW * k) + n16;
    const float bm = bias(A::LFC, j), bl = bias(A::LFC, Z + j);
    f32x4 z;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      mu[k][i] = acc[0][i] + bm;
      lv[k][i] = acc[1][i] + bl;
      const float sd = __expf(0.5f * lv[k][i]);
      z[i] = mu[k][i] + ep[k][i] * sd;
      // the KL term (:243) of these latents is summed in the decoder-L0 backward, which computes
      // exp(logvar) anyway (same expression, same per-lane order: the sum is bit-identical)
      if (TAP && 4 * q + i < nrows) {
        if (a.mu_out) a.mu_out[(size_t)(b0 + 4 * q + i) * Z + j] = mu[k][i];
        if (a.lv_out) a.lv_out[(size_t)(b0 + 4 * q + i) * Z + j] = lv[k][i];
      }
    }
    img2(IDC{}, j, to_bf4(z));
  }, scl(integral_constant<int, PL::sFC>{}));
  bar();
  {  // D0 → A0
    f32x4 acc[1];
    constexpr integral_constant<int, PL::sD0> sD0{};
    gemm<A, P, PL::sD0>(ring, opnd(sD0, IDC{}), acc, AR, wave, lane, NoSide{}, scl(sD0));
    img_copy<A::CLS ? A::Kp(A::LD0) : A::ZH, 0, 3>(DCAT, dst, XT(A::LD0), A::Kp(A::LD0), 0, b0);
    img2(IA0{}, n, relu(acc[0], bias(A::LD0, n), integral_constant<int, A::MD(0)>{}));
  }
  // decoder layers 1 .. ND-2 (input: D(i-1)'s output, A0 for odd i)
  sfor<1, ND - 1>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    bar();
    __bf16* const in = (i & 1) ? A0 : A1;
    f32x4 acc[1];
    constexpr integral_constant<int, PL::sD0 + i> sI{};
    using IIN = std::conditional_t<(i & 1), IA0, IA1>;
    using IOUT = std::conditional_t<(i & 1), IA1, IA0>;
    gemm<A, P, PL::sD0 + i>(ring, opnd(sI, IIN{}), acc, AR, wave, lane, NoSide{}, scl(sI));
    img_copy<H, 0, 1>(in, dst, XT(A::LD(i)), H, 0, b0);
    img2(IOUT{}, n, relu(acc[0], bias(A::LD(i), n), integral_constant<int, A::MD(i)>{}));
  });
  bar();
  __bf16* const DLIN = ((ND - 2) & 1) ? A1 : A0;  // input image of the last decoder layer
  {  // last decoder layer + conditional_vae_loss (:229-268) + dL/drecon, over x_rel in
     // place; one n-tile per group, its loss epilogue beside the next tile's stream
    constexpr int NG3 = PL::step(PL::sDL).NTL;
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const float cr = a.w_recon * 2.f;
    f32x2 sr2 = {0.f, 0.f};
    // per-lane parts of the epilogue's indices, feature f = 16t + n16 of n-tile t = wave + NW·g: the
    // image slot ioff(f, q) = 256t + ioff(n16, q) (its swizzle (f >> 2) & 3 = n16 >> 2 for every t)
    // and the bias 16t + n16 — lane bases plus compile-time LDS offsets; f mod D from the lane's
    // (16·wave + n16) mod D and the group's (16·NW·g) mod D
    __bf16* const XIL = XIN + ioff(n16, q) + 256 * wave;
    const float* const BIL = BIAS + A::bias_off(A::LDL) + 16 * wave + n16;
    const int dlane = (16 * wave + n16) % D;
    gemm_grouped<A, P, PL::sDL>(ring, opnd(integral_constant<int, PL::sDL>{}, std::conditional_t<((ND - 2) & 1), IA1, IA0>{}), AR, wave, lane, [&](auto gg, f32x4(&accs)[1]) {
      constexpr int g = decltype(gg)::value;
      if constexpr (g == 0) img_copy<H, 0, 1>(DLIN, dst, XT(A::LDL), H, 0, b0);
      if (!(NW * (g + 1) <= NG3 || wave + NW * g < NG3)) return;  // wave-uniform: tile past the output
      const int t = wave + NW * g;
      const f32x4 acc = accs[0];
      const int f = 16 * t + n16;
      f32x4 gi = {0.f, 0.f, 0.f, 0.f};
      if (f < I) {
        const float b = BIL[16 * NW * g];
        const f32x4 xr = from_bf4(*(const bf16x4*)(XIL + 256 * NW * g));
        const int dg = dlane + (16 * NW * g) % D, d = dg >= D ? dg - D : dg;
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
        if constexpr (TAP) {
          if (a.recon_out)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (4 * q + i < nrows) a.recon_out[(size_t)(b0 + 4 * q + i) * I + f] = r[i];
        }
        if (16 * t < D) {  // wave-uniform: only these n-tiles hold timestep-0 features
          const f32x4 df = {d01[0], d01[1], d23[0], d23[1]};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (4 * q + i >= nrows) continue;
            if (f < D && (d == 1 || d == 2) && use_start) {  // timestep 0
              s_start += df[i] * df[i];
              gi[i] += a.w_start * 2.f * df[i] * inv_2B;
            }
            if (d == 0 && f < D && use_time) {
              s_t0 += r[i] * r[i];
              gi[i] += a.w_time * 2.f * r[i] * inv_B;
            }
          }
        }
        if (d == 0) {
          const int s = f / D;
          *(f32x4*)(RCH0 + s * R + 4 * q) = r;
          *(f32x4*)(GD0 + s * R + 4 * q) = gi;
        }
      }
      *(bf16x4*)(XIL + 256 * NW * g) = to_bf4(gi);  // pad features f >= I: 0
    }, scl(integral_constant<int, PL::sDL>{}));
    s_recon += sr2[0] + sr2[1];
  }
  bar();
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
  bar();

  // ================================================================ backward
  // dL/drecon → gT(DL): rounds of its 16-B copy, over the decoder backward steps
  static_assert(XR <= ND - 1, "the dL/drecon copy runs over the decoder backward steps");
  {  // last decoder layer ᵀ: dL/d h_D(ND-2) = GL · W_DL, ReLU mask of D(ND-2) → A0
    f32x4 acc[1];
    dgemm(integral_constant<int, PL::sDLb>{}, XIN, acc);
    img_copy<Ip, 0, 1>(XIN, dst, GT(A::LDL), A::Np(A::LDL), 0, b0);
    img(A0, n, masked(acc[0], integral_constant<int, A::MD(ND - 2)>{}));
  }
  // D(i)ᵀ for i = ND-2 .. 1: input = dL/d(pre-activation of D(i)) = gT(D(i)), mask of D(i-1)
  sfor<1, ND - 1>([&](auto kk) {
    constexpr int k = decltype(kk)::value, i = ND - 1 - k;  // k-th decoder backward step after DLᵀ
    bar();
    __bf16* const in = (k & 1) ? A0 : A1;
    f32x4 acc[1];
    gemm<A, P, PL::sDLb + k>(ring, in, acc, AR, wave, lane);
    img_copy<H, 0, 1>(in, dst, GT(A::LD(i)), H, 0, b0);
    if constexpr (k < XR) img_copy<Ip, k, k + 1>(XIN, dst, GT(A::LDL), A::Np(A::LDL), 0, b0);
    img((k & 1) ? A1 : A0, n, masked(acc[0], integral_constant<int, A::MD(i - 1)>{}));
  });
  bar();
  // D0ᵀ: [dz ‖ dh_c(decoder share)]; dz → KL/reparameterisation backward → dL/d[mu ‖ logvar]
  __bf16* const D0IN = ((ND - 2) & 1) ? A1 : A0;  // gT(D0) image
  f32x4 dhc2;
  float* const DHC2 = (float*)(smem + A::L_DHC2);  // SZ only
  if constexpr (A::SZ) {  // tiles wave, wave + 8: features f < Z are dz, Z <= f < Z + H dh_c (to LDS)
    constexpr int TS = PL::step(PL::sD0b).TS, NTL = PL::step(PL::sD0b).NTL;
    f32x4 acc[TS];
    gemm<A, P, PL::sD0b>(ring, D0IN, acc, AR, wave, lane);
    img_copy<H, 0, 1>(D0IN, dst, GT(A::LD0), H, 0, b0);
    sfor<0, TS>([&](auto ss) {
      constexpr int s = decltype(ss)::value;
      const int t = wave + NW * s, f = 16 * t + n16;
      if (NW * (s + 1) > NTL && t >= NTL) return;  // wave-uniform: a reloaded tile
      if (f < Z) {
        const int j = f;
        f32x4 gm, gl;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool live = 4 * q + i < nrows;
          const float sd = __expf(0.5f * lv[0][i]);
          gm[i] = live ? a.w_kld * mu[0][i] * inv_BZ + acc[s][i] : 0.f;
          gl[i] = live ? a.w_kld * 0.5f * (__expf(lv[0][i]) - 1.f) * inv_BZ + acc[s][i] * ep[0][i] * 0.5f * sd : 0.f;
        }
        img(GFC, j, to_bf4(gm));
        img(GFC, Z + j, to_bf4(gl));
      } else if (f < A::ZH) {
        *(f32x4*)(DHC2 + (f - Z) * R + 4 * q) = acc[s];
      } else if (A::CLS && f < A::ZH + A::CLS_EMAX) {  // cfg4: the decoder's share of de
        *(f32x4*)((float*)(smem + A::L_DCE2) + (f - A::ZH) * R + 4 * q) = acc[s];
      }
    });
    // the fc-backward image's K padding (the region held the forward fc input until now)
    if (tid < (A::Np(A::LFC) - 2 * Z) * 4) *(uint64_t*)(GFC + (2 * Z + tid / 4) * 16 + 4 * (tid & 3)) = 0ull;
  } else {
    f32x4 acc[NZT + 1];
    dgemm(integral_constant<int, PL::sD0b>{}, D0IN, acc);
    img_copy<H, 0, 1>(D0IN, dst, GT(A::LD0), H, 0, b0);
#pragma unroll
    for (int k = 0; k < NZT; ++k) {
      const int j = 16 * (wave + NW * k) + n16;
      f32x4 gm, gl;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool live = 4 * q + i < nrows;
        const float sd = __expf(0.5f * lv[k][i]), el = __expf(lv[k][i]);
        if (live) s_kl += 1.f + lv[k][i] - mu[k][i] * mu[k][i] - el;  // KL (:243), from the fc epilogue
        gm[i] = live ? a.w_kld * mu[k][i] * inv_BZ + acc[k][i] : 0.f;
        gl[i] = live ? a.w_kld * 0.5f * (el - 1.f) * inv_BZ + acc[k][i] * ep[k][i] * 0.5f * sd : 0.f;
      }
      img(GFC, j, to_bf4(gm));
      img(GFC, Z + j, to_bf4(gl));
    }
    dhc2 = acc[NZT];  // feature n of dh_c: the lane that masks it in the fc backward
  }
  bar();
  {  // fcᵀ: dh = G_fc · W_fc → h_traj gradient (mask E(NE-1)) and h_c gradient (+ decoder share, mask C1)
    // CLS: tiles 16, 17 (waves 0, 1, slot 2) are de = fc share + decoder share (no activation) → gT(LCE)
    constexpr int TS = PL::step(PL::sFCb).TS;
    f32x4 acc[TS];
    dgemm(integral_constant<int, PL::sFCb>{}, GFC, acc);
    sub();
    img_copy<A::Np(A::LFC), 0, (2 * A::Np(A::LFC) + NT - 1) / NT>(GFC, dst, GT(A::LFC), A::Np(A::LFC), 0, b0);
    if constexpr (A::SZ) dhc2 = *(const f32x4*)(DHC2 + n * R + 4 * q);
    img(A0, n, masked(acc[0], integral_constant<int, A::ME(NE - 1)>{}));
    img(CB, n, masked(acc[1] + dhc2, integral_constant<int, A::MC1>{}));
    if constexpr (A::CLS) {
      static_assert(TS == 3 && A::Kp(A::LFC) == 2 * H + 32, "the class tiles are slot 2 of waves 0, 1");
      if (wave < 2) {  // wave-uniform
        const int k = 16 * wave + n16;
        f32x4 de = acc[2];
        if (k < A::CLS_EMAX) de += *(const f32x4*)((const float*)(smem + A::L_DCE2) + k * R + 4 * q);
        img((__bf16*)(smem + A::L_GCE), k, to_bf4(de));
      }
    }
  }
  // E(i)ᵀ for i = NE-1 .. 2 (input: gT(E(i)) image), mask of E(i-1)
  sfor<0, NE - 2>([&](auto kk) {
    constexpr int k = decltype(kk)::value, i = NE - 1 - k;
    bar();
    __bf16* const in = (k & 1) ? A1 : A0;
    f32x4 acc[1];
    gemm<A, P, PL::sFCb + 1 + k>(ring, in, acc, AR, wave, lane);
    img_copy<H, 0, 1>(in, dst, GT(A::LE(i)), H, 0, b0);
    if constexpr (k == 0) img_copy<H, 0, 1, 2 * H>(CB, dst, GT(A::LC1), H, 0, b0);
    if constexpr (A::CLS && k == 0)
      img_copy<A::Np(A::LCE), 1, 2, NT>((const __bf16*)(smem + A::L_GCE), dst, GT(A::LCE), A::Np(A::LCE), 0, b0);
    img((k & 1) ? A0 : A1, n, masked(acc[0], integral_constant<int, A::ME(i - 1)>{}));
  });
  bar();
  {  // E1ᵀ ‖ C1ᵀ: the last two gradients, gT(E0) and gT(C0), only feed the dW kernel
    __bf16* const in = ((NE - 2) & 1) ? A1 : A0;  // gT(E1) image
    __bf16* const oE = ((NE - 2) & 1) ? A0 : A1;  // free
    __bf16* const oC = GFC;                        // free (U region)
    f32x4 acc[1];
    gemm<A, P, PL::sC1b - 1>(ring, in, acc, AR, wave, lane);
    img_copy<H, 0, 1>(in, dst, GT(A::LE(1)), H, 0, b0);
    img(oE, n, masked(acc[0], integral_constant<int, A::ME(0)>{}));
    gemm<A, P, PL::sC1b>(ring, CB, acc, AR, wave, lane);
    img(oC, n, masked(acc[0], integral_constant<int, A::MC0>{}));
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
    bar();
    img_copy<H, 0, 1>(oE, dst, GT(A::LE0), H, 0, b0);
    img_copy<H, 0, 1, 2 * H>(oC, dst, GT(A::LC0), H, 0, b0);
  }
  if (tid < 5) {
    float s = 0.f;
    for (int w = 0; w < NW; ++w) s += PART[w * 8 + tid];
    __hip_atomic_store((unsigned*)(a.partials + blk * 8 + tid), __builtin_bit_cast(unsigned, s), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);  // (a plain store here took the cfg4 chain to 130 VGPRs)
  }
  if (CVAE_DIAG_STAMPS && a.stamps && tid < 64)
    gst<unsigned long long>(a.stamps + blk * 64 + tid, tid < stamp_i ? STAMPS[tid] : 0ull);
}

// BASELINE cfg5: S=200, D=6, latent 512, 8 + 8 layers (hidden 128)
using Cfg5 = Arch<200, 6, 512, 8, 8>;
// BASELINE cfg2 / the reference architecture: S=100, D=6, latent 8, 4 + 4 layers
using Cfg2 = Arch<100, 6, 8, 4, 4>;
// BASELINE cfg5 in the CVAE_FP8 form (e4m3 forward GEMMs; the large dX GEMMs e4m3 with MX scales)
using Cfg5F8 = Arch<200, 6, 512, 8, 8, true>;
// ... with every dX GEMM bf16 (CVAE_FP8_DX=bf16 at creation: the accuracy fallback and its A/B)
using Cfg5F8B = Arch<200, 6, 512, 8, 8, true, false, false>;
// BASELINE cfg4: the reference architecture at cfg2's shape with the scenario-class embedding
using Cfg4 = Arch<100, 6, 8, 4, 4, false, true>;
#ifndef CVAE_WIDE_RING
#define CVAE_WIDE_RING 12
#endif
constexpr int RING = CVAE_WIDE_RING;
#ifndef CVAE_RING_P
#define CVAE_RING_P 12
#endif

// ctr (the device step counters) rides in the preloaded kernel-argument SGPRs beside the x-tile
// arguments: read from RowArgs, the Philox-offset load waited for a kernel-argument fetch before
// the first x load could issue
template <class A, bool TAP = false, bool XB = false>
__global__ __launch_bounds__(NT) void widechain_kernel(char* arena, const void* x, const int64_t* idx, int Bp,
                                                       int batch, uint64_t* ctr, RowArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  RowArgs ra = a;
  ra.x = x;
  ra.idx = idx;
  ra.batch = batch;
  ra.ctr = ctr;
  wide_body<A, A::SZ ? CVAE_RING_P : RING, TAP, XB>(arena, Bp, ra, smem, blockIdx.x);
}

}  // namespace wchain
