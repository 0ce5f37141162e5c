// cvae_widewgrad.h — the dW ⊕ Adam kernel of BASELINE cfg5's wide shape (the wide chain's arena,
// wchain::Arch<200, 6, 512, 8, 8[, F8]>): wgrad_body over the same 32 × 64 / 32 × 32 tile list the
// generic wgrad_kernel<…, NI2> reads from memory, with the tile (layer, o0, i0, ni) and the layer
// record decoded from blockIdx and the Arch's compile-time layout instead.  The generic kernel's
// first operand load waits for three dependent round trips (kernel arguments → tile descriptor →
// layer record in the kernel arguments); here it waits for the preloaded scalar arguments only.
//
// Both decodings restate build_plan (cvae_capi.hip): the wide tile list (a layer whose padded K is a
// multiple of 64 takes 32 × 64 tiles, the others 32 × 32; layer by layer, the longer of Np / Kp
// outermost; the list cut into 8 contiguous chunks, chunk x at blockIdx 8j + x) and the flat
// parameter table (state_dict order, fc = fc_mu ‖ fc_logvar).  plan_wide checks both against the
// handle before enabling it.
#pragma once
#include "cvae_fastwgrad.h"
#include "cvae_widechain.h"

namespace wchain {

template <class A>
struct WTiles {
  static constexpr int NL = A::NL;
  __host__ __device__ static constexpr int ni(int l) { return A::Kp(l) % 64 == 0 && l != A::LCE ? 2 : 1; }
  __host__ __device__ static constexpr int count(int l) { return (A::Np(l) / 32) * (A::Kp(l) / (32 * ni(l))); }
  __host__ __device__ static constexpr int start(int l) {
    int t = 0;
    for (int k = 0; k < l; ++k) t += count(k);
    return t;
  }
  __host__ __device__ static constexpr int total() { return start(NL); }
  __host__ __device__ static constexpr int log2i(int v) { return v <= 1 ? 0 : 1 + log2i(v / 2); }
  __host__ __device__ static constexpr bool i_outer(int l) { return A::Kp(l) > A::Np(l); }
  __host__ __device__ static constexpr int inner(int l) { return i_outer(l) ? A::Np(l) / 32 : A::Kp(l) / (32 * ni(l)); }
  __host__ __device__ static constexpr bool pow2_inner() {
    for (int l = 0; l < NL; ++l)
      if (inner(l) & (inner(l) - 1)) return false;
    return true;
  }
  static_assert(pow2_inner(), "tile decode assumes power-of-two inner tile counts");
  // tile of workgroup b (host: the reference decode plan_wide compares with the handle's list)
  __host__ __device__ static TileDesc at(int b) {
    constexpr int NTL = total(), q = NTL / 8, r = NTL % 8;
    const int x = b & 7, j = b >> 3;
    const int s = x * q + (x < r ? x : r) + j;
#ifdef __HIP_DEVICE_COMPILE__
    int l = 0;
#pragma unroll
    for (int k = 1; k < NL; ++k) l += s >= start(k) ? 1 : 0;
    const int loc = s - (int)fchain::pick<NL>(l, [](int k) { return (int64_t)start(k); });
    const int sh = (int)fchain::pick<NL>(l, [](int k) { return (int64_t)log2i(inner(k)); });
    const bool io = fchain::pick<NL>(l, [](int k) { return (int64_t)i_outer(k); }) != 0;
    const int n = (int)fchain::pick<NL>(l, [](int k) { return (int64_t)ni(k); });
    const int a = loc >> sh, c = loc & ((1 << sh) - 1);
    return TileDesc{l, 32 * (io ? c : a), 32 * n * (io ? a : c), n};
#else
    int l = 0;
    while (l + 1 < NL && s >= start(l + 1)) ++l;
    const int loc = s - start(l), a = loc / inner(l), c = loc % inner(l);
    return TileDesc{l, 32 * (i_outer(l) ? c : a), 32 * ni(l) * (i_outer(l) ? a : c), ni(l)};
#endif
  }
};

// real in/out features of layer l of the Arch (Training_VAE.py:132-167, widened)
template <class A>
__host__ __device__ constexpr int wK(int l) {
  return l == A::LC0 ? 2 : l == A::LE0 ? A::I : l == A::LFC ? 2 * H : l == A::LD0 ? A::Z + H : H;
}
template <class A>
__host__ __device__ constexpr int wN(int l) {
  return l == A::LFC ? 2 * A::Z : l == A::LDL ? A::I : H;
}
// flat parameter offset of layer l: Σ_{k<l} (N_k·K_k + N_k) in state_dict order
template <class A>
__host__ __device__ constexpr int64_t wpoff(int l) {
  int64_t o = 0;
  for (int k = 0; k < l; ++k) o += (int64_t)wN<A>(k) * wK<A>(k) + wN<A>(k);
  return o;
}

// layer record of layer l (the fields build_plan / alloc_arena fill in)
template <class A>
__host__ __device__ inline LayerDev wide_layer(int l, char* arena, int Bp) {
#ifdef __HIP_DEVICE_COMPILE__
  auto P = [&](auto f) { return fchain::pick<A::NL>(l, f); };
#else
  auto P = [&](auto f) { return f(l); };
#endif
  static_assert(!A::CLS, "the class-embedding form's dW runs the generic kernel");
  LayerDev L{};
  L.K = (int)P([](int k) { return (int64_t)wK<A>(k); });
  L.N = (int)P([](int k) { return (int64_t)wN<A>(k); });
  L.Kp = (int)P([](int k) { return (int64_t)A::Kp(k); });
  L.Np = (int)P([](int k) { return (int64_t)A::Np(k); });
  L.relu = (l == A::LFC || l == A::LDL) ? 0 : 1;
  L.f8 = (int)P([](int k) { return (int64_t)A::f8(k); });
  L.f8b = (int)P([](int k) { return (int64_t)A::f8b(k); });
  L.wt = 0;
  L.has_bias = 1;
  const int64_t off = P([](int k) { return wpoff<A>(k); });
  const bool fc = l == A::LFC;  // fc_mu.weight, fc_mu.bias, fc_logvar.weight, fc_logvar.bias
  L.nseg = fc ? 2 : 1;
  L.seg_rows0 = fc ? A::Z : L.N;
  const int R0 = fc ? A::Z : L.N;
  L.pw[0] = off;
  L.pb[0] = off + (int64_t)R0 * L.K;
  L.pw[1] = fc ? L.pb[0] + A::Z : off;
  L.pb[1] = fc ? L.pw[1] + (int64_t)A::Z * L.K : L.pb[0];
  const int64_t Bp2 = 2 * (int64_t)Bp;
  L.Wf = arena + P([](int k) { return A::wf(k); });
  L.Wb = arena + P([](int k) { return A::wb(k); });
  L.Wb8 = L.f8b ? arena + P([](int k) { return A::f8b(k) ? A::wb8(k) : (int64_t)0; }) : nullptr;
  L.bias = (float*)(arena + A::bias_base) + P([](int k) { return (int64_t)A::bias_off(k); });
  L.xT = arena + A::act0 + Bp2 * P([](int k) { return A::xrows(k); });
  L.gT = arena + A::act0 + Bp2 * P([](int k) { return A::grows(k); });
  return L;
}

// grid = total tiles × sk.S + 1 (split-major; the last block finishes the loss).  Two workgroups per
// CU (4 waves per SIMD): the 436 tiles of cfg5 fit the 512 slots in one round.
// MXW: the 32 × 64 tiles' dW GEMMs in e4m3 with MX block scales along the batch (mx_dw_chunk,
// CVAE_FP8_DW=mx; Bk % 128 == 0); the 32 × 32 tiles (the K=2 condition layer) stay bf16
template <class A, int MODE, bool MXW = false>
__global__ __launch_bounds__(WG_THREADS, 4) void widewgrad_kernel(char* arena, float* params, float* mst, float* vst,
                                                                int Bp, int Bk, AdamArgs a, LossArgs la, SplitK sk) {
  AdamArgs aa = a;
  aa.params = params;
  aa.m = mst;
  aa.v = vst;
  constexpr int NTL = WTiles<A>::total();
  if ((int)blockIdx.x == NTL * sk.S) {  // one extra block finishes the loss beside the tiles
    if (threadIdx.x < 64 && la.partials) finish_loss(la, A::S, A::D, A::Z);
    return;
  }
  __shared__ __attribute__((aligned(16))) WgradLds<2> sh;
  sk.s = blockIdx.x / NTL;
  sk.tile = blockIdx.x - sk.s * NTL;
  const TileDesc td = WTiles<A>::at(sk.tile);
  const LayerDev L = wide_layer<A>(td.layer, arena, Bp);
  if (td.ni == 2)  // block-uniform
    wgrad_body<__bf16, MODE, 2, MXW>(L, td, Bk, aa, la, false, A::S, A::D, A::Z, sh.red, sh.dbp, sk);
  else
    wgrad_body<__bf16, MODE, 1>(L, td, Bk, aa, la, false, A::S, A::D, A::Z, sh.red, sh.dbp, sk);
}

// BASELINE cfg4 (A::CLS, the class embedding at the reference architecture's shape): the handle's
// list there is 32 × 32 tiles only (fewer than 512), in the same order (layer by layer, the longer
// of Np / Kp outermost, XCD chunks); the class-dependent widths — fc's input [h_traj ‖ h_c ‖ e] and
// decoder L0's [z ‖ h_c ‖ e] grow by class_dim, the table is n_classes × class_dim and the last
// parameter tensor — come from two runtime arguments.  plan_ring_cls checks the tile list and every
// layer record against the handle before enabling it (cvae_capi.hip cls_dw_matches).
template <class A>
struct CTiles {
  static constexpr int NL = A::NL;
  __host__ __device__ static constexpr int count(int l) { return (A::Np(l) / 32) * (A::Kp(l) / 32); }
  __host__ __device__ static constexpr int start(int l) {
    int t = 0;
    for (int k = 0; k < l; ++k) t += count(k);
    return t;
  }
  __host__ __device__ static constexpr int total() { return start(NL); }
  __host__ __device__ static constexpr int log2i(int v) { return v <= 1 ? 0 : 1 + log2i(v / 2); }
  __host__ __device__ static constexpr bool i_outer(int l) { return A::Kp(l) > A::Np(l); }
  __host__ __device__ static constexpr int inner(int l) { return i_outer(l) ? A::Np(l) / 32 : A::Kp(l) / 32; }
  __host__ __device__ static constexpr bool pow2_inner() {
    for (int l = 0; l < NL; ++l)
      if (inner(l) & (inner(l) - 1)) return false;
    return true;
  }
  static_assert(pow2_inner(), "tile decode assumes power-of-two inner tile counts");
  __host__ __device__ static TileDesc at(int b) {
    constexpr int NTL = total(), q = NTL / 8, r = NTL % 8;
    const int x = b & 7, j = b >> 3;
    const int s = x * q + (x < r ? x : r) + j;
#ifdef __HIP_DEVICE_COMPILE__
    int l = 0;
#pragma unroll
    for (int k = 1; k < NL; ++k) l += s >= start(k) ? 1 : 0;
    const int loc = s - (int)fchain::pick<NL>(l, [](int k) { return (int64_t)start(k); });
    const int sh = (int)fchain::pick<NL>(l, [](int k) { return (int64_t)log2i(inner(k)); });
    const bool io = fchain::pick<NL>(l, [](int k) { return (int64_t)i_outer(k); }) != 0;
    const int a = loc >> sh, c = loc & ((1 << sh) - 1);
    return TileDesc{l, 32 * (io ? c : a), 32 * (io ? a : c), 0};
#else
    int l = 0;
    while (l + 1 < NL && s >= start(l + 1)) ++l;
    const int loc = s - start(l), a = loc / inner(l), c = loc % inner(l);
    return TileDesc{l, 32 * (i_outer(l) ? c : a), 32 * (i_outer(l) ? a : c), 0};
#endif
  }
};

template <class A>
__host__ __device__ inline LayerDev cls_layer(int l, char* arena, int Bp, int ncls, int E) {
#ifdef __HIP_DEVICE_COMPILE__
  auto P = [&](auto f) { return fchain::pick<A::NL>(l, f); };
#else
  auto P = [&](auto f) { return f(l); };
#endif
  static_assert(A::CLS && !A::F8, "the class-embedding form (bf16)");
  LayerDev L{};
  const bool ce = l == A::LCE, fc = l == A::LFC;
  L.K = ce ? ncls : (int)P([](int k) { return (int64_t)wK<A>(k); }) + ((fc || l == A::LD0) ? E : 0);
  L.N = ce ? E : (int)P([](int k) { return (int64_t)wN<A>(k); });
  L.Kp = (int)P([](int k) { return (int64_t)A::Kp(k); });
  L.Np = (int)P([](int k) { return (int64_t)A::Np(k); });
  L.relu = (fc || l == A::LDL || ce) ? 0 : 1;
  L.wt = ce ? 1 : 0;
  L.has_bias = ce ? 0 : 1;
  // state_dict order with fc and decoder L0 widened by E; the table is the last tensor
  const int64_t off = P([](int k) { return wpoff<A>(k); }) + (l > A::LFC ? 2LL * A::Z * E : 0) +
                      (l > A::LD0 ? (int64_t)H * E : 0);
  L.nseg = fc ? 2 : 1;
  L.seg_rows0 = fc ? A::Z : L.N;
  const int R0 = fc ? A::Z : L.N;
  L.pw[0] = off;
  L.pb[0] = ce ? -1 : off + (int64_t)R0 * L.K;
  L.pw[1] = fc ? L.pb[0] + A::Z : off;
  L.pb[1] = fc ? L.pw[1] + (int64_t)A::Z * L.K : L.pb[0];
  const int64_t Bp2 = 2 * (int64_t)Bp;
  L.Wf = arena + P([](int k) { return A::wf(k); });
  L.Wb = arena + P([](int k) { return A::wb(k); });
  L.bias = (float*)(arena + A::bias_base) + P([](int k) { return (int64_t)A::bias_off(k); });
  L.xT = arena + A::act0 + Bp2 * P([](int k) { return A::xrows(k); });
  L.gT = arena + A::act0 + Bp2 * P([](int k) { return A::grows(k); });
  return L;
}

// grid = total tiles × sk.S + 1 (split-major; the last block finishes the loss)
template <class A, int MODE>
__global__ __launch_bounds__(WG_THREADS, 4) void clswgrad_kernel(char* arena, float* params, float* mst, float* vst,
                                                               int Bp, int Bk, int ncls, int E, AdamArgs a, LossArgs la,
                                                               SplitK sk) {
  AdamArgs aa = a;
  aa.params = params;
  aa.m = mst;
  aa.v = vst;
  constexpr int NTL = CTiles<A>::total();
  if ((int)blockIdx.x == NTL * sk.S) {
    if (threadIdx.x < 64 && la.partials) finish_loss(la, A::S, A::D, A::Z);
    return;
  }
  __shared__ __attribute__((aligned(16))) WgradLds<1> sh;
  sk.s = blockIdx.x / NTL;
  sk.tile = blockIdx.x - sk.s * NTL;
  const TileDesc td = CTiles<A>::at(sk.tile);
  const LayerDev L = cls_layer<A>(td.layer, arena, Bp, ncls, E);
  wgrad_body<__bf16, MODE, 1>(L, td, Bk, aa, la, false, A::S, A::D, A::Z, sh.red, sh.dbp, sk);
}

}  // namespace wchain
