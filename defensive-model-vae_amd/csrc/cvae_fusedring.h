// cvae_fusedring.h — one launch per training step for the reference architecture at S = 100
// (BASELINE cfg2: Training_VAE.py:345-363 — forward, conditional_vae_loss, backward, Adam): the
// single-ring row chain (cvae_widechain.h, blocks 0 .. nchain-1), every dW ⊕ Adam tile of
// fastwgrad_kernel (blocks nchain .. nchain+NTL-1) and the loss block, all resident at once — two
// workgroups per CU (<= 128 VGPRs, the chain's 65 KB of LDS; the tiles use the same dynamic LDS
// for their reduction image).  The tiles are dispatched with the chain, issue their fp32
// master-state loads at once and wait for the chain inside the launch: the boundary between the
// two launches and the dW launch's dispatch ramp overlap the chain instead of following it.
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup hand-off, sc1 form with a replicated counter):
// every chain block stores its arena rows, loss partials and (block 0) the step's counters and
// Adam scalars write-through (sc1), drains them (vmcnt(0)), joins a barrier, and ONE wave
// instruction adds 1 to each of the 8 replicas of the ready counter (a 128-B line each).  A tile
// block polls the replica of its XCD (one lane, sc1 loads, s_sleep) until it counts nchain; the
// block joins a barrier and reads the arena rows, partials and Adam scalars with sc1 loads only.
// The chain blocks never wait, so every wait ends; it is bounded anyway (~2 s of s_memrealtime):
// a time-out skips that block's update, sets the sticky flag and the handle's fault word, and the
// next training call fails (CVAE_E_TIMEOUT).
// Self-resetting counters: every tile block and the loss block add 1 to a done counter after
// their wait; the last resets the replicas and itself to zero — every chain add and every poll of
// this launch precede it — so no memset or counter kernel runs between steps.
#pragma once
#include "cvae_fastwgrad.h"
#include "cvae_widechain.h"

namespace wchain {

// the launch's hand-off words (cvae_capi.hip alloc_arena: 2 KB, zero between launches):
// [32 r] ready replica r (r < 8), [256] done counter, [288] sticky time-out flag
constexpr int RF_READY = 0, RF_DONE = 256, RF_FLAG = 288, RF_WORDS = 512;

struct RingFuseArgs {
  AdamArgs aa;
  LossArgs la;
  unsigned* sync;   // RF_* words
  unsigned* fault;  // the handle's fault word (pinned host memory)
  uint64_t timeout; // bound of a wait, s_memrealtime ticks (100 MHz)
  int Bk;           // batch rows rounded to the dW K chunk
  int nchain;       // row-chain blocks
};

// one lane of a block: wait until the block's replica counts f.nchain (sc1 loads, s_sleep between
// polls), then the whole block: returns false on a time-out (block-uniform)
struct ReadyGate {
  static constexpr bool gated = true;
  const RingFuseArgs* f;
  int* word;  // LDS
  __device__ bool operator()() const {
    if (threadIdx.x == 0) {
      const unsigned* rep = f->sync + RF_READY + 32 * (blockIdx.x & 7);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int ok = 1;
      while (__hip_atomic_load(rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)f->nchain) {
        __builtin_amdgcn_s_sleep(4);
        if (__builtin_amdgcn_s_memrealtime() - t0 > f->timeout) {
          __hip_atomic_store(f->sync + RF_FLAG, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (f->fault) __hip_atomic_store(f->fault, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          ok = 0;
          break;
        }
      }
      *word = ok;
    }
    __syncthreads();
    return *word != 0;
  }
};

#ifndef CVAE_FRING_P
#define CVAE_FRING_P 11  // 12 (the two-launch chain's depth) spills at 128 VGPRs
#endif

// grid = NTL + 1 blocks: block b < nchain runs row tile b of the chain, then (after the wait) dW
// tile NTL - nchain + b; block b >= nchain runs dW tile b - nchain; block NTL is the loss block.
// A chain block's CU thus takes one tile too, and the tile blocks alone spread over the other CUs
// (as the two-launch dW kernel's 280 blocks do): with a tile block per chain block on top, 89 CUs
// held two tiles and the dW tail grew (profiles/r03f).  Tile t keeps fastwgrad_kernel's XCD chunk
// (block index ≡ t mod 8 when nchain % 8 == 0).
template <class A>
__global__ __launch_bounds__(NT, 4) void fused_ring_kernel(char* arena, const void* x, const int64_t* idx, int Bp,
                                                          int batch, uint64_t* ctr, RowArgs a, RingFuseArgs f) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using TL = fchain::Tiles<19>;
  constexpr int NTL = TL::total();
  static_assert(sizeof(WgradLds<1>) + 16 <= A::L_TOTAL, "the tiles' reduction image fits the chain's LDS");
  // blocks nchain .. NTL-1: tiles 0 .. NTL-nchain-1; block NTL: the loss block (tb == NTL)
  int tb = (int)blockIdx.x == NTL ? NTL : (int)blockIdx.x - f.nchain;
  if ((int)blockIdx.x < f.nchain) {
    RowArgs ra = a;
    ra.x = x;
    ra.idx = idx;
    ra.batch = batch;
    ra.ctr = ctr;
    wide_body<A, CVAE_FRING_P>(arena, Bp, ra, smem, blockIdx.x, f.sync + RF_READY);
    __syncthreads();  // the chain's LDS becomes the tile's reduction image
    tb = NTL - f.nchain + (int)blockIdx.x;
  }
  WgradLds<1>* const sh = (WgradLds<1>*)smem;
  int* const word = (int*)(smem + sizeof(WgradLds<1>));
  const ReadyGate gate{&f, word};
  if (tb < NTL) {
    const fchain::FastNet fn{arena, Bp, A::S, A::D, A::I};
    TileDesc td;
    LayerDev L;
    fchain::decode_tile<19>(tb, fn.arena, fn.Bp, fn.I, td, L);
    wgrad_body<__bf16, PM_ADAM, true, 1>(L, td, f.Bk, f.aa, f.la, false, A::S, A::D, A::Z, sh->red, sh->dbp,
                                         SplitK{1, 0, nullptr, nullptr, tb, 0}, nullptr, gate);
  } else if (gate() && threadIdx.x < 64 && f.la.partials) {  // the loss block
    finish_loss<true>(f.la, A::S, A::D, A::Z);
  }
  // every block past its wait: the last resets the counters for the next launch
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(f.sync + RF_DONE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)NTL) {  // NTL tiles + the loss block
#pragma unroll
      for (int r = 0; r < 8; ++r) __hip_atomic_store(f.sync + RF_READY + 32 * r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(f.sync + RF_DONE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace wchain
