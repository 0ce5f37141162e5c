// cvae_fastwgrad.h — the dW ⊕ Adam kernel of the fast configuration (the one fastchain_kernel
// serves): the same wgrad_body as the generic wgrad_kernel, with the tile (layer, o0, i0) and the
// layer record derived from blockIdx and the compile-time arena layout instead of read from memory.
// A generic block's first operand load waits for three dependent round trips (kernel arguments →
// tile descriptor → layer record in the kernel arguments); here it waits for one.
//
// Both decodings restate build_plan (cvae_capi.hip): tile order (layer by layer, the longer of
// Np/Kp outermost, the list cut into 8 contiguous chunks and chunk x placed at blockIdx 8j + x) and
// the flat parameter table (state_dict order, fc = fc_mu ‖ fc_logvar).  plan_fast checks both
// against the handle's tables before enabling the fast path.
#pragma once
#include "cvae_fastchain.h"
#include "cvae_wgrad.h"

namespace fchain {

// real in/out features of layer l (I = seq_len · dim)
__host__ __device__ constexpr int fK(int l, int I) {
  return l == LC0 ? 2 : l == LE0 ? I : l == LFC ? 2 * H : l == LD0 ? Z + H : H;
}
__host__ __device__ constexpr int fN(int l, int I) { return l == LFC ? 2 * Z : l == LD3 ? I : H; }

// value f(l) of a compile-time function at a runtime layer index: a chain of scalar selects
// (branch-free; the block's decode runs before its first load, and branches there cost fetches)
template <int NL, typename F>
__device__ __forceinline__ int64_t pick(int l, F f) {
  int64_t v = f(0);
#pragma unroll
  for (int k = 1; k < NL; ++k) v = l == k ? f(k) : v;
  return v;
}

template <int NKI>
struct Tiles {
  using LY = Layout<NKI>;
  // input tiles per workgroup (wgrad_body<NI>).  NI = 2 for D3 (38 tiles of 32 × 64 instead of
  // 76, 243 workgroups: one per CU) measured no faster than 280 workgroups with 24 CUs doubled
  // (7.18 vs 7.23 µs): a 64-wide tile costs what two co-resident tiles do.  Kept at 1.
  __host__ __device__ static constexpr int ni(int) { return 1; }
  __host__ __device__ static constexpr int ni_max() {
    int m = 1;
    for (int l = 0; l < LY::NL; ++l) m = ni(l) > m ? ni(l) : m;
    return m;
  }
  __host__ __device__ static constexpr int count(int l) { return (LY::Np(l) / 32) * (LY::Kp(l) / (32 * ni(l))); }
  __host__ __device__ static constexpr int start(int l) {
    int t = 0;
    for (int k = 0; k < l; ++k) t += count(k);
    return t;
  }
  __host__ __device__ static constexpr int total() { return start(LY::NL); }
  __host__ __device__ static constexpr int log2i(int v) { return v <= 1 ? 0 : 1 + log2i(v / 2); }
  // the divisor of a layer's tile index (the inner tile count) is a power of two for this
  // architecture: the decode is shifts and masks
  __host__ __device__ static constexpr bool i_outer(int l) { return LY::Kp(l) > LY::Np(l); }
  __host__ __device__ static constexpr int inner(int l) {
    return i_outer(l) ? LY::Np(l) / 32 : LY::Kp(l) / (32 * ni(l));
  }
  __host__ __device__ static constexpr bool pow2_inner() {
    for (int l = 0; l < LY::NL; ++l)
      if (inner(l) & (inner(l) - 1)) return false;
    return true;
  }
  static_assert(pow2_inner(), "tile decode assumes power-of-two inner tile counts");
  // list position of workgroup b in a launch over n consecutive list entries (xcd_order: the n
  // cut into 8 contiguous chunks, chunk x at blockIdx 8j + x)
  __host__ __device__ static int slot(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7, j = b >> 3;
    return x * q + (x < r ? x : r) + j;
  }
  // tile of workgroup b (host: the reference decode plan_fast compares with the handle's list)
  __host__ __device__ static TileDesc at(int b) { return decode(slot(b, total())); }
  // the two dW buckets (CVAE_PART_DW_DEC / _REST): the decoder layers are the list's tail
  __host__ __device__ static constexpr int bucket_first(int k) { return k == 0 ? start(LD0) : 0; }
  __host__ __device__ static constexpr int bucket_count(int k) { return k == 0 ? total() - start(LD0) : start(LD0); }
  // tile at list position s
  __host__ __device__ static TileDesc decode(int s) {
#ifdef __HIP_DEVICE_COMPILE__
    int l = 0;
#pragma unroll
    for (int k = 1; k < LY::NL; ++k) l += s >= start(k) ? 1 : 0;
    const int loc = s - (int)pick<LY::NL>(l, [](int k) { return (int64_t)start(k); });
    const int sh = (int)pick<LY::NL>(l, [](int k) { return (int64_t)log2i(inner(k)); });
    const bool io = pick<LY::NL>(l, [](int k) { return (int64_t)i_outer(k); }) != 0;
    const int w = 32 * (int)pick<LY::NL>(l, [](int k) { return (int64_t)ni(k); });  // input width
    const int a = loc >> sh, c = loc & ((1 << sh) - 1);
    return TileDesc{l, 32 * (io ? c : a), w * (io ? a : c), 0};
#else
    int l = 0;
    while (l + 1 < LY::NL && s >= start(l + 1)) ++l;
    const int loc = s - start(l), a = loc / inner(l), c = loc % inner(l);
    return TileDesc{l, 32 * (i_outer(l) ? c : a), 32 * ni(l) * (i_outer(l) ? a : c), 0};
#endif
  }
};

// layer record of layer l (the fields build_plan / alloc_arena fill in).  Flat parameter offset of
// layer l = Σ_{k<l} (N_k·K_k + N_k); only E0 (K = I) precedes a layer with an I-dependent term.
template <int NKI>
__host__ __device__ constexpr int64_t poff_const(int l) {
  int64_t o = 0;
  for (int k = 0; k < l; ++k) o += k == LE0 ? (int64_t)H : (int64_t)fN(k, 0) * fK(k, 0) + fN(k, 0);
  return o;
}

template <int NKI>
__host__ __device__ inline LayerDev fast_layer(int l, char* arena, int Bp, int I) {
  using LY = Layout<NKI>;
#ifdef __HIP_DEVICE_COMPILE__
  auto P = [&](auto f) { return pick<LY::NL>(l, f); };
#else
  auto P = [&](auto f) { return f(l); };
#endif
  LayerDev L{};
  const int K = l == LE0 ? I : (int)P([](int k) { return (int64_t)fK(k, 0); });
  const int N = l == LD3 ? I : (int)P([](int k) { return (int64_t)fN(k, 0); });
  L.K = K;
  L.N = N;
  L.Kp = (int)P([](int k) { return (int64_t)LY::Kp(k); });
  L.Np = (int)P([](int k) { return (int64_t)LY::Np(k); });
  L.relu = (l == LFC || l == LD3) ? 0 : 1;
  L.has_bias = 1;
  const int64_t off = P([](int k) { return poff_const<NKI>(k); }) + (l > LE0 ? (int64_t)H * I : 0);
  const bool fc = l == LFC;  // fc_mu.weight, fc_mu.bias, fc_logvar.weight, fc_logvar.bias
  L.nseg = fc ? 2 : 1;
  L.seg_rows0 = fc ? Z : N;
  const int R0 = fc ? Z : N;
  L.pw[0] = off;
  L.pb[0] = off + (int64_t)R0 * K;
  L.pw[1] = fc ? L.pb[0] + Z : off;
  L.pb[1] = fc ? L.pw[1] + (int64_t)Z * K : L.pb[0];
  const int64_t Bp2 = 2 * (int64_t)Bp;
  L.Wf = arena + P([](int k) { return LY::wf(k); });
  L.Wb = arena + P([](int k) { return LY::wb(k); });
  L.bias = (float*)(arena + LY::bias_base) + P([](int k) { return (int64_t)LY::bias_off(k); });
  L.xT = arena + LY::act0 + Bp2 * P([](int k) { return LY::xrows(k); });
  L.gT = arena + LY::act0 + Bp2 * P([](int k) { return LY::grows(k); });
  return L;
}

// The tile and its layer record (compile-time decode: scalar selects, no memory round trip).
// Measured alternative (round 3): wave 0 decodes and broadcasts the record through LDS +
// readfirstlane, cutting the kernel's SALU instructions ~8x — no faster (dW 7.8 vs 7.7-7.9 µs,
// profiles/r03d): the scalar issue is not what the tiles wait on.
template <int NKI>
__device__ __forceinline__ void decode_tile(int tile, char* arena, int Bp, int I, TileDesc& td, LayerDev& L) {
  td = Tiles<NKI>::at(tile);
  L = fast_layer<NKI>(td.layer, arena, Bp, I);
}

// Scalars first (SGPR-preloaded at wave launch, as fastchain_kernel's): the arena and master-state
// pointers every first load needs.
// grid = total tiles × sk.S + 1 (split-major; the last block finishes the loss)
template <int NKI, int MODE>
__global__ __launch_bounds__(WG_THREADS) void fastwgrad_kernel(char* arena, float* params, float* mst, float* vst,
                                                                int Bp, int Bk, int S, int D, int I, AdamArgs a,
                                                                LossArgs la, SplitK sk) {
  const FastNet fn{arena, Bp, S, D, I};
  AdamArgs aa = a;
  aa.params = params;
  aa.m = mst;
  aa.v = vst;
  constexpr int NTL = Tiles<NKI>::total();
  if ((int)blockIdx.x == NTL * sk.S) {  // one extra block finishes the loss beside the tiles
    if (threadIdx.x < 64 && la.partials) finish_loss(la, fn.S, fn.D, Z);
    return;
  }
  __shared__ __attribute__((aligned(16))) WgradLds<Tiles<NKI>::ni_max()> sh;
  sk.s = blockIdx.x / NTL;
  sk.tile = blockIdx.x - sk.s * NTL;
  TileDesc td;
  LayerDev L;
  decode_tile<NKI>(sk.tile, fn.arena, fn.Bp, fn.I, td, L);
  if (Tiles<NKI>::ni(td.layer) == 2)  // block-uniform
    wgrad_body<__bf16, MODE, 2>(L, td, Bk, aa, la, false, fn.S, fn.D, Z, sh.red, sh.dbp, sk);
  else
    wgrad_body<__bf16, MODE, 1>(L, td, Bk, aa, la, false, fn.S, fn.D, Z, sh.red, sh.dbp, sk);
}

// One dW bucket of the data-parallel two-bucket step (dist.py buckets=2): the tiles of list
// positions [first, first + n) — Tiles::bucket_first/count — in the same XCD placement the generic
// kernel's bucket lists (build_plan tiles_part) have.  grid = n × sk.S + 1; the last block
// finishes the loss when the call carries it (the decoder bucket, launched with the chain).
// Split-K tickets and partials are indexed by the list position, so the two buckets never share one.
template <int NKI, int MODE>
__global__ __launch_bounds__(WG_THREADS) void fastwgrad_bucket_kernel(char* arena, float* params, float* mst,
                                                                       float* vst, int Bp, int Bk, int S, int D, int I,
                                                                       AdamArgs a, LossArgs la, SplitK sk, int first,
                                                                       int n) {
  const FastNet fn{arena, Bp, S, D, I};
  AdamArgs aa = a;
  aa.params = params;
  aa.m = mst;
  aa.v = vst;
  if ((int)blockIdx.x == n * sk.S) {
    if (threadIdx.x < 64 && la.partials) finish_loss(la, fn.S, fn.D, Z);
    return;
  }
  static_assert(Tiles<NKI>::ni_max() == 1, "bucket tiles are 32 x 32");
  __shared__ __attribute__((aligned(16))) WgradLds<1> sh;
  sk.s = blockIdx.x / n;
  sk.tile = first + Tiles<NKI>::slot((int)blockIdx.x - sk.s * n, n);
  const TileDesc td = Tiles<NKI>::decode(sk.tile);
  const LayerDev L = fast_layer<NKI>(td.layer, fn.arena, fn.Bp, fn.I);
  wgrad_body<__bf16, MODE, 1>(L, td, Bk, aa, la, false, fn.S, fn.D, Z, sh.red, sh.dbp, sk);
}

// Adam from the all-reduced gradient buffer (the RCCL data-parallel step's last launch,
// cvae_adam): param_kernel's body over fastwgrad's tiles, the tile and layer record decoded from
// blockIdx instead of read from the tile list and the NetDev kernel argument (two dependent round
// trips before the first state load).  grid = Tiles::total(), CVAE_THREADS threads.
template <int NKI>
__global__ __launch_bounds__(CVAE_THREADS) void fastadam_kernel(char* arena, float* params, float* mst, float* vst,
                                                                const float* grads, int Bp, int I, AdamArgs a) {
  __shared__ __attribute__((aligned(16))) float wt[32 * WT_LD];
  AdamArgs aa = a;
  aa.params = params;
  aa.m = mst;
  aa.v = vst;
  aa.grads = const_cast<float*>(grads);
  TileDesc td;
  LayerDev L;
  decode_tile<NKI>(blockIdx.x, arena, Bp, I, td, L);
  param_body<__bf16, PM_ADAM>(L, td, aa, wt);
}

// ---------------------------------------------------------------- data parallel: the peer exchange
// fastwgrad_kernel's tiles with cvae_peer.h's exchange: tile b is owned by rank b mod world (its
// block runs the Adam epilogue and broadcasts the operand copies), every other rank's block for b
// pushes its partial to the owner.  The last block finishes this rank's loss, then waits until
// every tile the other ranks own has arrived (px.n_remote per step).
// grid = G + 1: tile block b takes tiles b, b + G, b + 2G, .. — every one it PUSHES first, then the
// ones it OWNS (the only ones that wait).  One rank per GPU: G = tiles (one tile per block, every
// block resident: 281 blocks in 512 slots).  Ranks sharing a GPU (cvae_px_import counts them): G is
// cut so that Σ over those ranks of max(row-chain blocks, G + 1) <= the GPU's workgroup slots (two
// per CU at <= 128 VGPRs and these LDS sizes) — every block of every sharing rank can then be
// resident at once, so a waiting owner never holds a slot a pusher of another rank needs, and no
// push waits at all (cvae_peer.h, residency precondition).
// SHARED = false: one tile per block (G = tiles); true: the loop over tiles b, b + G, .. (ranks
// sharing a GPU — a rehearsal, not the measured path)
template <int NKI, bool SHARED = false>
__global__ __launch_bounds__(WG_THREADS, 4) void px_wgrad_kernel(char* arena, float* params, float* mst, float* vst,
                                                               int Bp, int Bk, int S, int D, int I, AdamArgs a,
                                                               LossArgs la, PeerArgs px) {
  const FastNet fn{arena, Bp, S, D, I};
  AdamArgs aa = a;
  aa.params = params;
  aa.m = mst;
  aa.v = vst;
  constexpr int NTL = Tiles<NKI>::total();
  const int G = SHARED ? (int)gridDim.x - 1 : NTL;
  if ((int)blockIdx.x == G) {
    if (threadIdx.x < 64 && la.partials) finish_loss(la, fn.S, fn.D, Z);
    if (threadIdx.x == 0)
      px_wait(px_done(px, px.mbox[px.rank]), (uint64_t)px.n_remote * px_epoch(px, aa.ctr), px.fault, px.timeout, 3,
              px_stats(px), 1);
    return;
  }
  __shared__ __attribute__((aligned(16))) WgradLds<1> sh;
  static_assert(Tiles<NKI>::ni_max() == 1, "the exchange's partial is one 32 x 32 tile");
  auto tile = [&](int t, bool owned) {
    SplitK sk{1, 0, nullptr, nullptr, t, 0};
    TileDesc td;
    LayerDev L;
    decode_tile<NKI>(t, fn.arena, fn.Bp, fn.I, td, L);
    if (owned)
      wgrad_body<__bf16, PM_ADAM, 1>(L, td, Bk, aa, la, false, fn.S, fn.D, Z, sh.red, sh.dbp, sk, &px);
    else
      wgrad_body<__bf16, PM_GRAD, 1>(L, td, Bk, aa, la, false, fn.S, fn.D, Z, sh.red, sh.dbp, sk, &px);
  };
  if constexpr (!SHARED) {
    tile(blockIdx.x, px_owner(blockIdx.x, px.world) == px.rank);  // block-uniform
  } else {
#pragma nounroll
    for (int owned = 0; owned < 2; ++owned) {  // pushes first, then the owner tiles (which wait)
#pragma nounroll
      for (int t = blockIdx.x; t < NTL; t += G) {
        if ((px_owner(t, px.world) == px.rank) != (owned == 1)) continue;  // block-uniform
        __syncthreads();  // several tiles per block: the previous one's LDS is free
        tile(t, owned == 1);
      }
    }
  }
}

}  // namespace fchain
