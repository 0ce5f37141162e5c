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
  // tile of workgroup b (host: the reference decode plan_fast compares with the handle's list)
  __host__ __device__ static TileDesc at(int b) {
    constexpr int NTL = total(), q = NTL / 8, r = NTL % 8;
    const int x = b & 7, j = b >> 3;
    const int s = x * q + (x < r ? x : r) + j;
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
    wgrad_body<__bf16, MODE, false, 2>(L, td, Bk, aa, la, false, fn.S, fn.D, Z, sh.red, sh.dbp, sk);
  else
    wgrad_body<__bf16, MODE, false, 1>(L, td, Bk, aa, la, false, fn.S, fn.D, Z, sh.red, sh.dbp, sk);
}

// ---------------------------------------------------------------- data parallel: the peer exchange
// fastwgrad_kernel's tiles with cvae_peer.h's exchange: tile b is owned by rank b mod world (its
// block runs the Adam epilogue and broadcasts the operand copies), every other rank's block for b
// pushes its partial to the owner.  The last block finishes this rank's loss, then waits until
// every tile the other ranks own has arrived (px.n_remote per step).  grid = tiles + 1.
// Two workgroups per CU (4 waves per SIMD, <= 128 VGPRs): every block of the launch is resident at
// once with room to spare, so waiting owner blocks can never hold the slots their pushers need —
// also when several ranks share one GPU (tests/test_gpu_peer.py).
template <int NKI>
__global__ __launch_bounds__(WG_THREADS, 4) void px_wgrad_kernel(char* arena, float* params, float* mst, float* vst,
                                                               int Bp, int Bk, int S, int D, int I, AdamArgs a,
                                                               LossArgs la, PeerArgs px) {
  const FastNet fn{arena, Bp, S, D, I};
  AdamArgs aa = a;
  aa.params = params;
  aa.m = mst;
  aa.v = vst;
  constexpr int NTL = Tiles<NKI>::total();
  if ((int)blockIdx.x == NTL) {
    if (threadIdx.x < 64 && la.partials) finish_loss(la, fn.S, fn.D, Z);
    if (threadIdx.x == 0)
      px_wait(px_done(px, px.mbox[px.rank]), (uint64_t)px.n_remote * px_epoch(px, aa.ctr), px.fault, px.timeout, 3,
              px_stats(px), 1);
    return;
  }
  __shared__ __attribute__((aligned(16))) WgradLds<1> sh;
  SplitK sk{1, 0, nullptr, nullptr, (int)blockIdx.x, 0};
  TileDesc td;
  LayerDev L;
  decode_tile<NKI>(sk.tile, fn.arena, fn.Bp, fn.I, td, L);
  static_assert(Tiles<NKI>::ni_max() == 1, "the exchange's partial is one 32 x 32 tile");
  if (px_owner(sk.tile, px.world) == px.rank)  // block-uniform
    wgrad_body<__bf16, PM_ADAM, false, 1>(L, td, Bk, aa, la, false, fn.S, fn.D, Z, sh.red, sh.dbp, sk, &px);
  else
    wgrad_body<__bf16, PM_GRAD, false, 1>(L, td, Bk, aa, la, false, fn.S, fn.D, Z, sh.red, sh.dbp, sk, &px);
}

// ---------------------------------------------------------------- the fused training step
// One launch = the row chain (blocks 0 .. nchain-1) and every dW ⊕ Adam tile (blocks nchain ..).
// The tiles are listed in the order their arena rows become final (chain_body's groups), so the
// tile blocks resident beside the chain are the ones its backward pass releases first: the
// decoder's and fc's dW overlap the encoder's backward steps instead of following the whole chain,
// and the launch boundary between the two kernels disappears.
//   group 0 (after S11): D0 D1 D2 | group 1 (after S13): D3 FC E3 C1 | group 2 (end): E2 E1 E0 C0
// Visibility (MI355X_MICROARCH.md, inter-workgroup hand-off, sc1 form): the chain stores every
// arena row and loss partial sc1 and drains them before its per-group agent-scope add; a tile
// block polls its group's counter (one lane, relaxed sc1 loads, bounded), joins a workgroup
// barrier, then reads the rows with sc1 loads only.  Deadlock-free: tiles wait only on chain
// blocks, which have the lowest indices and are dispatched first; the spin gives up after ~0.5 s
// (flag sync[4]; the tile then skips its update) rather than hang.  The host zeroes the counters
// before every launch (stream-ordered memset).
__host__ __device__ constexpr int ready_layer(int k) {
  return k == 0 ? LD0 : k == 1 ? LD1 : k == 2 ? LD2 : k == 3 ? LD3 : k == 4 ? LFC : k == 5 ? LE3
       : k == 6 ? LC1 : k == 7 ? LE2 : k == 8 ? LE1 : k == 9 ? LE0 : LC0;
}
__host__ __device__ constexpr int ready_group(int l) {
  return (l == LD0 || l == LD1 || l == LD2) ? 0 : (l == LD3 || l == LFC || l == LE3 || l == LC1) ? 1 : 2;
}

template <int NKI>
struct ReadyTiles {
  using T = Tiles<NKI>;
  static constexpr int NL = Layout<NKI>::NL;
  __host__ __device__ static constexpr int start(int k) {
    int t = 0;
    for (int j = 0; j < k; ++j) t += T::count(ready_layer(j));
    return t;
  }
  __host__ __device__ static TileDesc at(int tb) {
#ifdef __HIP_DEVICE_COMPILE__
    int k = 0;
#pragma unroll
    for (int j = 1; j < NL; ++j) k += tb >= start(j) ? 1 : 0;
    const int l = (int)pick<NL>(k, [](int j) { return (int64_t)ready_layer(j); });
    const int loc = tb - (int)pick<NL>(k, [](int j) { return (int64_t)start(j); });
    const int sh = (int)pick<NL>(k, [](int j) { return (int64_t)T::log2i(T::inner(ready_layer(j))); });
    const bool io = pick<NL>(k, [](int j) { return (int64_t)T::i_outer(ready_layer(j)); }) != 0;
    const int w = 32 * (int)pick<NL>(k, [](int j) { return (int64_t)T::ni(ready_layer(j)); });
    const int a = loc >> sh, c = loc & ((1 << sh) - 1);
#else
    int k = 0;
    while (k + 1 < NL && tb >= start(k + 1)) ++k;
    const int l = ready_layer(k), loc = tb - start(k), a = loc / T::inner(l), c = loc % T::inner(l);
    const bool io = T::i_outer(l);
    const int w = 32 * T::ni(l);
#endif
    return TileDesc{l, 32 * (io ? c : a), w * (io ? a : c), 0};
  }
};

struct FusedArgs {
  AdamArgs aa;
  LossArgs la;
  unsigned* sync;  // [0..2] group counters (zeroed by the host before the launch), [3] unused, [4] sticky spin time-out flag
  unsigned* fault; // the handle's fault word (pinned host memory): set on a time-out, fails the next training call
  int Bk;          // batch rows rounded to the dW K chunk
  int nchain;      // row-chain blocks
};

#ifndef FUSED_SLEEP
#define FUSED_SLEEP 32
#endif
template <int NKI>
__global__ __launch_bounds__(NT) void fused_step_kernel(FastNet fn, RowArgs a, FusedArgs f) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((int)blockIdx.x < f.nchain) {
    chain_body<NKI>(fn, a, smem, f.sync, blockIdx.x);
    return;
  }
  constexpr int NTL = Tiles<NKI>::total();
  const int tb = blockIdx.x - f.nchain;
  const TileDesc td = ReadyTiles<NKI>::at(tb);
#ifdef FUSED_DIAG  // diagnostic builds: 1 = tiles exit at once, 2 = tiles exit after their wait
  if (FUSED_DIAG == 1) return;
#endif
  // one lane polls its group's counter (bounded); on a time-out the tile sets the sticky flag
  // sync[4] and SKIPS its update (reading unfinished rows would corrupt params, m and v), so a
  // failed step leaves the old parameters of its tiles and cvae_sync_words reports it
  __shared__ int timed_out;
  if (threadIdx.x == 0) {
    unsigned* cnt = f.sync + ready_group(td.layer);
    int to = 0;
    for (unsigned spins = 0;
         __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)f.nchain;) {
      __builtin_amdgcn_s_sleep(FUSED_SLEEP);  // ~FUSED_SLEEP·64 cycles: ~200 pollers must not load the fabric
      if (++spins == (1u << 24) / FUSED_SLEEP) {
        __hip_atomic_store(f.sync + 4, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f.fault) __hip_atomic_store(f.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        to = 1;
        break;
      }
    }
    timed_out = to;
  }
  __syncthreads();
  if (timed_out) return;
#ifdef FUSED_DIAG
  if (FUSED_DIAG == 2) return;
#endif
  const LayerDev L = fast_layer<NKI>(td.layer, fn.arena, fn.Bp, fn.I);
  __shared__ __attribute__((aligned(16))) WgradLds<Tiles<NKI>::ni_max()> sh;
  if (Tiles<NKI>::ni(td.layer) == 2)
    wgrad_body<__bf16, PM_ADAM, true, 2>(L, td, f.Bk, f.aa, f.la, tb == NTL - 1, fn.S, fn.D, Z, sh.red, sh.dbp);
  else
    wgrad_body<__bf16, PM_ADAM, true, 1>(L, td, f.Bk, f.aa, f.la, tb == NTL - 1, fn.S, fn.D, Z, sh.red, sh.dbp);
  // the group counters are zeroed by the host before every fused launch (hipMemsetAsync on the
  // same stream), never inside the kernel: a reset here could race chain blocks still adding
}

}  // namespace fchain
