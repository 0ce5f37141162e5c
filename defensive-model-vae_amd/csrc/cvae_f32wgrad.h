// cvae_f32wgrad.h — the dW ⊕ Adam launch of the fp32 chain's configuration (f32c::Arch: the
// reference's own shape, Training_VAE.py:274-282, :362-363): the generic wgrad_body<float> per
// 32 × 32 tile, with the tile (layer, o0, i0) and the layer record derived from blockIdx and the
// compile-time arena layout instead of read from memory (as cvae_fastwgrad.h does for the bf16
// reference architecture at S = 100).  The generic kernel's first operand load waits for the tile
// descriptor (global memory) and then the layer record (kernel arguments, indexed by the tile's
// layer); here both are scalar selects on blockIdx.
//
// Tile order: layer by layer, the longer of Np/Kp outermost, the list cut into 8 contiguous chunks
// and chunk x placed at blockIdx 8j + x (one XCD's L2 then fetches few layers' rows).  Every tile is
// one independent wgrad_body call, so the order does not change a bit of the result; plan_f32c
// checks that the decode covers the handle's tile list exactly and that every layer record equals
// the handle's before enabling it.
#pragma once
#include "cvae_f32chain.h"
#include "cvae_fastwgrad.h"

namespace f32c {

template <class A>
struct WTiles {
  static constexpr int count(int l) { return (A::Np(l) / 32) * (A::Kp(l) / 32); }
  static constexpr int start(int l) {
    int t = 0;
    for (int k = 0; k < l; ++k) t += count(k);
    return t;
  }
  static constexpr int total() { return start(NL); }
  static constexpr int log2i(int v) { return v <= 1 ? 0 : 1 + log2i(v / 2); }
  static constexpr bool i_outer(int l) { return A::Kp(l) > A::Np(l); }
  static constexpr int inner(int l) { return i_outer(l) ? A::Np(l) / 32 : A::Kp(l) / 32; }
  static constexpr bool pow2_inner() {
    for (int l = 0; l < NL; ++l)
      if (inner(l) & (inner(l) - 1)) return false;
    return true;
  }
  static_assert(pow2_inner(), "the decode is shifts and masks");
  __host__ __device__ static int slot(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7, j = b >> 3;
    return x * q + (x < r ? x : r) + j;
  }
  __host__ __device__ static TileDesc at(int b) { return decode(slot(b, total())); }
  __host__ __device__ static TileDesc decode(int s) {
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

// layer record of layer l, as build_plan / alloc_arena fill it for fp32 operands (4-byte elements)
template <class A>
__host__ __device__ inline LayerDev f32_layer(int l, char* arena, int Bp) {
#ifdef __HIP_DEVICE_COMPILE__
  auto P = [&](auto f) { return fchain::pick<NL>(l, f); };
#else
  auto P = [&](auto f) { return f(l); };
#endif
  constexpr int I = A::I;
  LayerDev L{};
  L.K = (int)P([](int k) { return (int64_t)fchain::fK(k, I); });
  L.N = (int)P([](int k) { return (int64_t)fchain::fN(k, I); });
  L.Kp = (int)P([](int k) { return (int64_t)A::Kp(k); });
  L.Np = (int)P([](int k) { return (int64_t)A::Np(k); });
  L.relu = (l == LFC || l == LD3) ? 0 : 1;
  L.has_bias = 1;
  const int64_t off = P([](int k) { return fchain::poff_const<1>(k) + (k > LE0 ? (int64_t)H * I : 0); });
  const bool fc = l == LFC;  // fc_mu.weight, fc_mu.bias, fc_logvar.weight, fc_logvar.bias
  L.nseg = fc ? 2 : 1;
  L.seg_rows0 = fc ? Z : L.N;
  const int R0 = fc ? Z : L.N;
  L.pw[0] = off;
  L.pb[0] = off + (int64_t)R0 * L.K;
  L.pw[1] = fc ? L.pb[0] + Z : off;
  L.pb[1] = fc ? L.pw[1] + (int64_t)Z * L.K : L.pb[0];
  const int64_t Bp4 = 4 * (int64_t)Bp;
  L.Wf = arena + P([](int k) { return A::wf(k); });
  L.Wb = arena + P([](int k) { return A::wb(k); });
  L.bias = (float*)(arena + A::bias_base) + P([](int k) { return (int64_t)A::bias_off(k); });
  L.xT = arena + A::act0 + Bp4 * P([](int k) { return A::xrows(k); });
  L.gT = arena + A::act0 + Bp4 * P([](int k) { return A::grows(k); });
  return L;
}

// grid = total tiles × sk.S + 1 (split-major; the last block finishes the loss beside the tiles)
template <class A, int MODE>
__global__ __launch_bounds__(WG_THREADS) void f32wgrad_kernel(char* arena, float* params, float* mst, float* vst,
                                                              int Bp, int Bk, AdamArgs a, LossArgs la, SplitK sk) {
  AdamArgs aa = a;
  aa.params = params;
  aa.m = mst;
  aa.v = vst;
  constexpr int NTL = WTiles<A>::total();
  if ((int)blockIdx.x == NTL * sk.S) {
    if (threadIdx.x < 64 && la.partials) finish_loss(la, A::S, A::D, Z);
    return;
  }
  __shared__ __attribute__((aligned(16))) WgradLds<1> sh;
  sk.s = blockIdx.x / NTL;
  sk.tile = blockIdx.x - sk.s * NTL;
  const TileDesc td = WTiles<A>::at(sk.tile);
  const LayerDev L = f32_layer<A>(td.layer, arena, Bp);
  wgrad_body<float, MODE, 1>(L, td, Bk, aa, la, false, A::S, A::D, Z, sh.red, sh.dbp, sk);
}

}  // namespace f32c
