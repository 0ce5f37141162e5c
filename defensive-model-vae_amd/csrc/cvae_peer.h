// cvae_peer.h — the data-parallel exchange over xGMI without a collective library: dW ⊕
// reduce-scatter ⊕ Adam ⊕ all-gather inside the weight-gradient launch (the step the
// reference takes once per batch at Training_VAE.py:362-363, here across N ranks).
//
// Every rank computes every 32 × 32 dW tile over its own rows (its share of the global batch).
// Tile t belongs to rank owner(t) = t mod N (the launch's block index: with N = 8 that is the
// XCD chunk, 35 tiles each at the reference architecture).  Per step:
//   * a tile block on a NON-owner rank pushes its fp32 partial (32 × 32 dW + 32 db, 4.2 KB) into
//     the owner's mailbox slot [t][rank] with stores over xGMI, releases them at system scope and
//     adds 1 to the owner's flag[t];
//   * the OWNER's block for t computes its own partial, waits until flag[t] has counted N − 1
//     arrivals for this step, sums the N partials in rank order (the global-batch gradient up to
//     summation order, identical on every run), applies torch's Adam to its fp32 master p/m/v
//     (only the owner's copy of tile t is ever current) and writes the new operand copies
//     (Wf / Wb fragments and the fp32 bias) into its own arena AND every peer's arena, then adds
//     1 to every peer's done counter;
//   * one extra block per rank (the loss block) waits until its done counter has counted every
//     tile the other ranks own, so the launch ends only when this rank's operand copies are
//     complete: the next row chain reads them after the kernel boundary.
// Bytes per link and step at N = 8: 35 partials in + 35 tiles' Wf/Wb out ≈ 2 × 140 KB.
// Deadlock-free: non-owner blocks never wait, owners wait only on other ranks' non-owner blocks
// and the loss block only on owners; every wait is bounded (CVAE_PX_TIMEOUT_MS of s_memrealtime,
// default 10 s) and a time-out sets the handle's fault word and skips the update (cvae_fault; the
// next training call fails; cvae_px_reset re-arms the mailbox after the state is made whole).
// Residency precondition: a waiting owner holds a workgroup slot, so every pusher must find one
// without waiting for a waiter to finish.  One rank per GPU: the 281 blocks of a launch fit the
// 512 slots (two per CU).  k ranks sharing a GPU: Σ over them of max(row-chain blocks, exchange
// blocks) <= 512 — cvae_px_import counts the ranks on each GPU (PCI address in the blobs), gives
// each 512/k − 1 tile blocks (each pushing all its tiles before it waits on any it owns) and
// refuses a configuration whose row chain alone exceeds 512/k blocks.  Round 3's 4-rank stall
// (281 blocks per rank, 1,124 against 512 slots) ran without this bound.
// Mailboxes are uncached fine-grained allocations mapped into every rank through IPC;
// flags and counters are system-scope atomics; ragged global batches weight the partials by
// c_r = B_r / B_global, equal shares sum and then scale by 1/N (the RCCL path's grad_scale).
#pragma once
#include "cvae_device.h"

constexpr int PX_MAX = 16;                 // ranks
constexpr int PX_SLOTS_PER_CU = 2;         // workgroups of the row chain / exchange launch one CU holds

// CVAE_PX_SC (default): the partials' hand-off without cache maintenance — the system-scope
// analogue of MI355X_MICROARCH.md's sc1 form: every partial store write-through at system scope
// (sc0 sc1), every storing wave drains them, a barrier, ONE relaxed system-scope flag add; the
// owner polls with relaxed system-scope loads and reads the partials with sc0 sc1 loads.  0: a
// system-scope release fence (L2 write-back) per pushing block and acquire loads / an acquire fence
// on the owner — the split-K ticket with the agent-scope form of those fences ran 10x slower at
// B = 16384 (profiles/r03i).  The owner's broadcast of the new operand copies keeps its release.
#ifndef CVAE_PX_SC
#define CVAE_PX_SC 1
#endif
// 4- or 8-B pieces of a partial: system-scope relaxed atomic stores / loads (sc0 sc1)
template <typename V>
__device__ __forceinline__ void px_st(float* dst, V v) {
  static_assert(sizeof(V) % 8 == 0, "partial vectors of 8 or 16 B");
#pragma unroll
  for (int c = 0; c < (int)(sizeof(V) / 8); ++c) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 h = f2{v[2 * c], v[2 * c + 1]};
    __hip_atomic_store((uint64_t*)dst + c, __builtin_bit_cast(uint64_t, h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
template <typename V>
__device__ __forceinline__ V px_ld(const float* src) {
  V v;
#pragma unroll
  for (int c = 0; c < (int)(sizeof(V) / 8); ++c) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 h = __builtin_bit_cast(f2, __hip_atomic_load((const uint64_t*)src + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    v[2 * c] = h[0];
    v[2 * c + 1] = h[1];
  }
  return v;
}
constexpr int PX_PW = 32 * 32 + 32;        // floats of one tile's partial: dW [32][32], then db [32]

struct PeerArgs {
  int world, rank;
  int ragged;            // 0: g = (Σ_r g_r) · grad_scale (AdamArgs); 1: g = Σ_r c[r] · g_r
  int n_remote;          // tiles the other ranks own (done-counter arrivals per step)
  float c[PX_MAX];       // B_r / B_global (ragged)
  char* arena[PX_MAX];   // every rank's arena base, this rank's included (operand-copy destinations)
  char* mbox[PX_MAX];    // every rank's mailbox: flags [ntiles] u64 | done u64 | inbox [ntiles][world][PX_PW]
  int64_t done_off, inbox_off;
  uint64_t base;         // counters[1] when the exchange was set up (the same on every rank)
  unsigned* fault;       // the handle's fault word (pinned host memory)
  uint64_t timeout;      // bound of every wait, in s_memrealtime ticks (100 MHz)
};

// this rank's wait statistics, in its own mailbox after the done counter (cvae_px_stats):
// [0] max owner-tile wait, [1] max end-of-launch wait, [2] Σ owner-tile waits, [3] owner waits,
// all in s_memrealtime ticks (10 ns)
constexpr int PX_STATS_OFF = 256;

__host__ __device__ inline int px_owner(int tile, int world) { return tile % world; }

__device__ __forceinline__ uint64_t* px_flag(char* mb, int tile) { return (uint64_t*)mb + tile; }
__device__ __forceinline__ uint64_t* px_done(const PeerArgs& p, char* mb) { return (uint64_t*)(mb + p.done_off); }
__device__ __forceinline__ float* px_inbox(const PeerArgs& p, char* mb, int tile, int src) {
  return (float*)(mb + p.inbox_off) + ((size_t)tile * p.world + src) * PX_PW;
}

// one lane: wait until *w >= target (system-scope acquire loads), at most `timeout` ticks of
// s_memrealtime (100 MHz); on a time-out set the fault word to `code` and return false.  stats:
// this rank's statistics words (or null), `kind` 0 = owner tile, 1 = end of launch
__device__ __forceinline__ bool px_wait(const uint64_t* w, uint64_t target, unsigned* fault, uint64_t timeout,
                                        unsigned code = 2, uint64_t* stats = nullptr, int kind = 0) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t dt = 0;
  while (__hip_atomic_load(w, CVAE_PX_SC ? __ATOMIC_RELAXED : __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
    __builtin_amdgcn_s_sleep(4);
    dt = __builtin_amdgcn_s_memrealtime() - t0;
    if (dt > timeout) {
      if (fault) __hip_atomic_store(fault, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
  if (stats) {
    __hip_atomic_fetch_max(stats + kind, dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (kind == 0) {
      __hip_atomic_fetch_add(stats + 2, dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(stats + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  return true;
}
__device__ __forceinline__ uint64_t* px_stats(const PeerArgs& p) {
  return (uint64_t*)(p.mbox[p.rank] + p.done_off + PX_STATS_OFF);
}

// the step's epoch (1, 2, ... since set-up): the row chain that began the step advanced counters[1]
__device__ __forceinline__ uint64_t px_epoch(const PeerArgs& p, const uint64_t* ctr) { return ctr[1] - p.base; }

// non-owner: this block's partial (every thread EPT weights of row o at iv; threads < 32 the bias)
// into the owner's inbox, released at system scope, then one arrival on the owner's flag
template <typename V>
__device__ __forceinline__ void px_push(const PeerArgs& p, int tile, int o, int iv, V g, float db, bool bias_tile) {
  const int tid = threadIdx.x, owner = px_owner(tile, p.world);
  float* dst = px_inbox(p, p.mbox[owner], tile, p.rank);
  if (CVAE_PX_SC) {
    px_st(dst + o * 32 + iv, g);
    if (bias_tile && tid < 32)
      __hip_atomic_store((unsigned*)(dst + 1024 + tid), __builtin_bit_cast(unsigned, db), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every piece in the owner's memory before the flag
  } else {
    *(V*)(dst + o * 32 + iv) = g;
    if (bias_tile && tid < 32) dst[1024 + tid] = db;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the partial is in the owner's memory first
  }
  __syncthreads();
  if (tid == 0) __hip_atomic_fetch_add(px_flag(p.mbox[owner], tile), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// owner: wait for the N − 1 other partials of this step, sum all N in rank order.  Returns false
// (block-uniform) on a time-out: the caller then skips the update.
template <typename V>
__device__ __forceinline__ bool px_gather(const PeerArgs& p, const uint64_t* ctr, int tile, int o, int iv, V& g,
                                          float& db, bool bias_tile, int* ok_lds) {
  const int tid = threadIdx.x;
  if (tid == 0)
    *ok_lds = px_wait(px_flag(p.mbox[p.rank], tile), (uint64_t)(p.world - 1) * px_epoch(p, ctr), p.fault, p.timeout, 2,
                      px_stats(p), 0) ? 1 : 0;
  __syncthreads();
  if (!*ok_lds) return false;
  if (!CVAE_PX_SC) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  V s = {};
  float sb = 0.f;
  for (int r = 0; r < p.world; ++r) {
    V v;
    float vb = 0.f;
    if (r == p.rank) {
      v = g;
      vb = db;
    } else {
      const float* src = px_inbox(p, p.mbox[p.rank], tile, r);
      if (CVAE_PX_SC) {
        v = px_ld<V>(src + o * 32 + iv);
        if (bias_tile && tid < 32)
          vb = __builtin_bit_cast(float, __hip_atomic_load((const unsigned*)(src + 1024 + tid), __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_SYSTEM));
      } else {
        v = *(const V*)(src + o * 32 + iv);
        if (bias_tile && tid < 32) vb = src[1024 + tid];
      }
    }
    if (p.ragged) {
      v = v * p.c[r];
      vb = vb * p.c[r];
    }
    s = r == 0 ? v : s + v;
    sb = r == 0 ? vb : sb + vb;
  }
  g = s;
  db = sb;
  return true;
}
