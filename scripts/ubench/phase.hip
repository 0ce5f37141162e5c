// Microbenchmark (GPU box): one row-chain "step" structure in isolation, 64 workgroups, NSTEP steps
// of a 16-row × 128 × 128 bf16 layer per workgroup, every step reading a fresh 32-KB weight block
// (the same lines in every workgroup, 1 MB of distinct weights in all) and writing a 4-KB
// activation block to global memory.
//   A  (current design): 8 waves; each wave loads its own weight fragments into registers two
//      steps ahead and stores its 8-B-per-lane results itself.
//   B<L> (loader waves): 8 compute waves read weights from a 2-slot LDS ring; L extra loader waves
//      stage the weights global→registers→LDS (LA steps ahead in registers) and copy each finished
//      activation image LDS→global with 16-B stores.  Everyone meets at one s_barrier per step.
// Prints ns per step (difference of two step counts: launch overhead cancels).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
#define G __attribute__((address_space(1)))
#define LDSP __attribute__((address_space(3)))

constexpr int WSTEP = 32 * 1024;  // weight bytes per step per workgroup
constexpr int NWSTEPS = 96;       // distinct weight blocks (3 MB: every step of a launch reads fresh lines)

__device__ __forceinline__ void lbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ bf16x8 xfrag(const __bf16* img, int kc) {
  const int lane = threadIdx.x & 63;
  const int f = kc * 32 + 4 * (lane >> 4) + ((lane & 15) >> 2);
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDSP i16x4*)(img + f * 16 + 4 * (lane & 3)));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDSP i16x4*)(img + (f + 16) * 16 + 4 * (lane & 3)));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// ---- A: current design.  MODE bit0: no weight loads, bit1: no global stores; NB register sets
// (weights loaded NB-1 steps ahead)
template <int MODE, int NB>
__global__ __launch_bounds__(512) void kA(const __bf16* W, __bf16* out, int nstep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto img = [&](int i) { return (__bf16*)(smem + (i & 1) * 4096); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, n16 = lane & 15, q = lane >> 4;
  const int n = wave * 16 + n16;
  if (tid < 512) ((u32x4*)smem)[tid] = u32x4{0, 0, 0, 0};
  bf16x8 w[NB][4];
  auto wl = [&](bf16x8* wr, int s) {
    const __bf16* p = W + (size_t)(s % NWSTEPS) * (WSTEP / 2) + ((size_t)wave * 4 * 64 + lane) * 8;
#pragma unroll
    for (int c = 0; c < 4; ++c) wr[c] = (MODE & 1) ? bf16x8{} : *(const G bf16x8*)(p + c * 512);
  };
#pragma unroll
  for (int b = 0; b < NB - 1; ++b) wl(w[b], b);
  lbar();
  for (int s0 = 0; s0 < nstep; s0 += NB) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int s = s0 + b;
      const __bf16* in = img(s);
      __bf16* o = img(s + 1);
      const bool first = (MODE & 4) || ((MODE & 8) && (wave & 1));  // 8: odd waves first (staggered)
      if (first) wl(w[(b + NB - 1) % NB], s + NB - 1);
      bf16x8 x[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) x[c] = xfrag(in, c);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[c], w[b][c], acc, 0, 0, 0);
      bf16x4 h;
#pragma unroll
      for (int i = 0; i < 4; ++i) h[i] = (__bf16)fmaxf(acc[i] * 0.01f, 0.f);
      *(bf16x4*)(o + n * 16 + 4 * q) = h;
      if ((MODE & 16) && wave < 4) {  // half the waves store the step's 4 KB as 16-B pieces
        const u32x4 v = {(unsigned)acc[0], (unsigned)acc[1], (unsigned)acc[2], (unsigned)acc[3]};
        *(G u32x4*)((char*)out + (((size_t)blockIdx.x * nstep + s) * 2048) * 2 + (wave * 64 + lane) * 16) = v;
      } else if (!(MODE & 2) && !(MODE & 16)) {
        *(G bf16x4*)(out + ((size_t)blockIdx.x * nstep + s) * 2048 + n * 16 + 4 * q) = h;
      }
      if (!first) wl(w[(b + NB - 1) % NB], s + NB - 1);
      lbar();
    }
  }
}

// ---- E: the step's B operand from a resident LDS weight image (the decoder layers'
// forward fragments kept in LDS and read transposed for their dX instead of streaming the Wᵀ copy).
// The 32-KB image holds 8 n-tiles × [128 K-features][16 columns] bf16 in the activation-image layout
// (row quad q of feature f at slot q ^ ((f >> 2) & 3)), so a wave's fragment of chunk c is two
// ds_read_b64_tr_b16 — the same transposed read as its X operand.  MODE bit1: no global stores.
template <int MODE>
__global__ __launch_bounds__(512) void kE(const __bf16* W, __bf16* out, int nstep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto img = [&](int i) { return (__bf16*)(smem + (i & 1) * 4096); };
  const __bf16* wimg = (const __bf16*)(smem + 8192);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, n16 = lane & 15, q = lane >> 4;
  const int n = wave * 16 + n16;
  if (tid < 512) ((u32x4*)smem)[tid] = u32x4{0, 0, 0, 0};
  for (int i = tid; i < 32768 / 16; i += 512) ((u32x4*)(smem + 8192))[i] = *(const G u32x4*)((const char*)W + i * 16);
  lbar();
  for (int s = 0; s < nstep; ++s) {
    const __bf16* in = img(s);
    __bf16* o = img(s + 1);
    bf16x8 x[4], w[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = xfrag(in, c);
#pragma unroll
    for (int c = 0; c < 4; ++c) w[c] = xfrag(wimg + wave * 2048, c);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[c], w[c], acc, 0, 0, 0);
    bf16x4 h;
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = (__bf16)fmaxf(acc[i] * 0.01f, 0.f);
    *(bf16x4*)(o + n * 16 + 4 * q) = h;
    if (!(MODE & 2)) *(G bf16x4*)(out + ((size_t)blockIdx.x * nstep + s) * 2048 + n * 16 + 4 * q) = h;
    lbar();
  }
}

// ---- B: loader waves
template <int L, int LA>
__global__ __launch_bounds__(64 * (8 + L)) void kB(const __bf16* W, __bf16* out, int nstep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem + 8192;  // 2 × 32 KB
  auto img = [&](int i) { return (__bf16*)(smem + (i & 1) * 4096); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 512) ((u32x4*)smem)[tid] = u32x4{0, 0, 0, 0};
  constexpr int FPW = WSTEP / 1024 / L;  // fragments per loader wave per step
  if (wave >= 8) {
    const int lw = wave - 8;
    u32x4 r[LA][FPW];
    auto gl = [&](u32x4* d, int s) {
      const char* p = (const char*)W + (size_t)(s % NWSTEPS) * WSTEP + (size_t)lw * FPW * 1024 + lane * 16;
#pragma unroll
      for (int f = 0; f < FPW; ++f) d[f] = *(const G u32x4*)(p + f * 1024);
    };
    auto dw = [&](const u32x4* d, int s) {
      char* p = ring + (s & 1) * WSTEP + lw * FPW * 1024 + lane * 16;
#pragma unroll
      for (int f = 0; f < FPW; ++f) *(u32x4*)(p + f * 1024) = d[f];
    };
    // prologue: slot 0 filled, steps 1..LA in registers
    gl(r[0], 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dw(r[0], 0);
#pragma unroll
    for (int a = 0; a < LA; ++a) gl(r[a], 1 + a);
    lbar();
    for (int s0 = 0; s0 < nstep; s0 += LA) {
#pragma unroll
      for (int a = 0; a < LA; ++a) {
        const int s = s0 + a;
        // step s: write weights of step s+1 (oldest registers) into the free slot, reload them
        // with step s+1+LA, copy the image finished in step s-1 (img(s)) to global
        if (LA == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (LA == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FPW) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * FPW) : "memory");
        dw(r[a], s + 1);
        gl(r[a], s + 1 + LA);
        if (s > 0) {
          const int e = lw * 64 + lane;  // 16-B pieces of the 4-KB image: 256
          if (e < 256) {
            const u32x4 v = *(const u32x4*)((const char*)img(s) + e * 16);
            *(G u32x4*)((char*)out + (((size_t)blockIdx.x * nstep + s - 1) * 2048) * 2 + e * 16) = v;
          }
        }
        lbar();
      }
    }
    return;
  }
  const int n16 = lane & 15, q = lane >> 4, n = wave * 16 + n16;
  lbar();
  for (int s = 0; s < nstep; ++s) {
    const __bf16* in = img(s);
    __bf16* o = img(s + 1);
    const char* slot = ring + (s & 1) * WSTEP + wave * 4 * 1024 + lane * 16;
    bf16x8 x[4], w[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) w[c] = *(const bf16x8*)(slot + c * 1024);
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = xfrag(in, c);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[c], w[c], acc, 0, 0, 0);
    bf16x4 h;
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = (__bf16)fmaxf(acc[i] * 0.01f, 0.f);
    *(bf16x4*)(o + n * 16 + 4 * q) = h;
    lbar();
  }
}

// rewrites the weights from 256 workgroups (as the dW/Adam kernel does between row-chain launches):
// the next launch finds them in no L2
__global__ void rewrite(u32x4* W, int n16, unsigned v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) W[i] = u32x4{v, v, v, v};
}

// ---- C: one loader wave streams the weights by LDS-DMA into an NS-slot ring and never joins a
// barrier; the 8 compute waves synchronise through LDS counters instead of s_barrier.
__device__ __forceinline__ bool spin_ge(volatile unsigned* c, unsigned target, unsigned* err) {
  for (unsigned it = 0; *c < target; ++it) {
    __builtin_amdgcn_s_sleep(1);
    if (it > (1u << 22)) {
      err[0] = 1;
      return false;
    }
  }
  return true;
}
template <int NS, int MODE, int L = 1>  // MODE bit1: no global stores; L loader waves
__global__ __launch_bounds__(64 * (8 + L)) void kC(const __bf16* W, __bf16* out, int nstep, unsigned* err) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem + 8192;
  volatile unsigned* ctr = (volatile unsigned*)(smem + 8192 + NS * WSTEP);  // [0] ready steps, [1] done waves
  auto img = [&](int i) { return (__bf16*)(smem + (i & 1) * 4096); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 512) ((u32x4*)smem)[tid] = u32x4{0, 0, 0, 0};
  if (tid == 0) {
    ctr[0] = 0;
    ctr[1] = 0;
  }
  __syncthreads();
  if (wave >= 8) {
    constexpr int FPL = 32 / L;  // 1-KB pieces per loader wave per step
    const int lw = wave - 8;
    for (int s = 0; s < nstep; ++s) {
      if (s >= NS && !spin_ge(ctr + 1, 8u * (s - NS + 1), err)) return;
      const char* src = (const char*)W + (size_t)(s % NWSTEPS) * WSTEP + lw * FPL * 1024 + lane * 16;
      LDSP char* dst = (LDSP char*)ring + (s % NS) * WSTEP + lw * FPL * 1024;
#pragma unroll
      for (int f = 0; f < FPL; ++f)
        __builtin_amdgcn_global_load_lds((const G void*)(src + f * 1024), (LDSP void*)(dst + f * 1024), 16, 0, 0);
      if (s >= 1) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FPL) : "memory");  // step s-1 landed
        if (lane == 0) __hip_atomic_fetch_add((unsigned*)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add((unsigned*)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return;
  }
  const int n16 = lane & 15, q = lane >> 4, n = wave * 16 + n16;
  for (int s = 0; s < nstep; ++s) {
    if (!spin_ge(ctr, (unsigned)L * (s + 1), err)) return;
    const __bf16* in = img(s);
    __bf16* o = img(s + 1);
    const char* slot = ring + (s % NS) * WSTEP + wave * 4 * 1024 + lane * 16;
    bf16x8 x[4], w[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) w[c] = *(const bf16x8*)(slot + c * 1024);
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = xfrag(in, c);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[c], w[c], acc, 0, 0, 0);
    bf16x4 h;
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = (__bf16)fmaxf(acc[i] * 0.01f, 0.f);
    *(bf16x4*)(o + n * 16 + 4 * q) = h;
    if (!(MODE & 2)) *(G bf16x4*)(out + ((size_t)blockIdx.x * nstep + s) * 2048 + n * 16 + 4 * q) = h;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add((unsigned*)(ctr + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (!spin_ge(ctr + 1, 8u * (s + 1), err)) return;
  }
}

// ---- D<K>: the N-split chain (VERDICT r04 Next #6).  K co-XCD workgroups share one 16-row tile:
// member m computes outputs [m·128/K, (m+1)·128/K) of every step with 8/K waves, so each streams 1/K
// of the step's 32 KB of fragments, and the members exchange their activation slices through the
// XCD's L2 after every step: sc1 (write-through) stores of the slice, every storing wave's
// vmcnt(0), a barrier, one lane's agent-scope add to the tile's counter (MI355X_MICROARCH.md hand-off
// table, first row), one lane's sc1 poll until all K members have added, a barrier, then sc1 loads
// of the other members' slices into the LDS image.  Blocks 8·(K·(t/8) + m) + t%8 are tile t's
// members: all on XCD t % 8.  MODE bit1: no arena stores (the chain's 4-KB store per step);
// bit2: no exchange (the members run unsynchronised: the stream-only part of the price).
// Every spin is bounded (err[0] counts give-ups), so every wave reaches the end.
__device__ __forceinline__ bool spin_sc1(const unsigned* c, unsigned target, unsigned* err) {
  for (unsigned it = 0; __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++it) {
    __builtin_amdgcn_s_sleep(1);
    if (it > (1u << 22)) {
      atomicAdd(err, 1u);
      return false;
    }
  }
  return true;
}
template <int K, int MODE>
__global__ __launch_bounds__(512) void kD(const __bf16* W, __bf16* out, int nstep, unsigned* ctr, __bf16* xch,
                                          unsigned* err) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto img = [&](int i) { return (__bf16*)(smem + (i & 1) * 4096); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, n16 = lane & 15, q = lane >> 4;
  const int b = blockIdx.x, x = b % 8, j = b / 8, m = j % K, t = (j / K) * 8 + x;
  constexpr int WPM = 8 / K;           // computing waves per member
  constexpr int SL = 128 / K;          // features per member slice
  const bool comp = wave < WPM;
  const int n = m * SL + wave * 16 + n16;  // this lane's output feature (computing waves)
  if (tid < 512) ((u32x4*)smem)[tid] = u32x4{0, 0, 0, 0};
  bf16x8 w[3][4];
  auto wl = [&](bf16x8* wr, int s) {
    const __bf16* p = W + (size_t)(s % NWSTEPS) * (WSTEP / 2) + ((size_t)(m * WPM + wave) * 4 * 64 + lane) * 8;
#pragma unroll
    for (int c = 0; c < 4; ++c) wr[c] = *(const G bf16x8*)(p + c * 512);
  };
  if (comp) {
    wl(w[0], 0);
    wl(w[1], 1);
  }
  lbar();
  unsigned* my = ctr + t * 64;  // one counter per tile, on a line of its own
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(xch, (short)0, 0x7fffffff, 0x00020000);
  for (int s0 = 0; s0 < nstep; s0 += 3) {
#pragma unroll
    for (int bb = 0; bb < 3; ++bb) {
      const int s = s0 + bb;
      if (s >= nstep) break;
      const __bf16* in = img(s);
      __bf16* o = img(s + 1);
      if (comp) {
        bf16x8 xf[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) xf[c] = xfrag(in, c);
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[c], w[bb][c], acc, 0, 0, 0);
        bf16x4 h;
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = (__bf16)fmaxf(acc[i] * 0.01f, 0.f);
        *(bf16x4*)(o + n * 16 + 4 * q) = h;
        if (!(MODE & 4))  // the slice to the other members: 8 B per lane, write-through (sc1 = aux 16)
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h), xr,
                                                (int)((((size_t)t * 2 + (s & 1)) * 2048 + n * 16 + 4 * q) * 2), 0, 16);
        if (!(MODE & 2))  // the chain's arena copy of the step (its share of it)
          *(G bf16x4*)(out + ((size_t)t * nstep + s) * 2048 + n * 16 + 4 * q) = h;
        wl(w[(bb + 2) % 3], s + 2);
        if (!(MODE & 4)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // the slice stores (the 4 loads stay)
      }
      if (!(MODE & 4)) {
        __syncthreads();
        if (tid == 0) {
          __hip_atomic_fetch_add(my, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          spin_sc1(my, (unsigned)K * (s + 1), err);
        }
        __syncthreads();
        // the other members' slices: 16 rows × (128 − SL) features, 16-B sc1 loads into the image
        const int pieces = (128 - SL) * 16 * 2 / 16;  // 16-B pieces
        for (int e = tid; e < pieces; e += 512) {
          const int fo = e / 2, half = e & 1;           // feature among the others, row half
          const int f = fo < m * SL ? fo : fo + SL;     // skip this member's own slice
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
              xr, (int)((((size_t)t * 2 + (s & 1)) * 2048 + f * 16 + half * 8) * 2), 0, 16);  // sc1 load
          *(u32x4*)((char*)o + (f * 16 + half * 8) * 2) = v;
        }
      }
      lbar();
    }
  }
}

template <typename F>
float timeit(F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) launch();
  const int reps = 30;
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e6f / reps;  // ns per launch
}

int main(int argc, char** argv) {
  const bool only_d = argc > 1 && argv[1][0] == 'D';
  __bf16 *W, *out;
  hipMalloc(&W, (size_t)WSTEP * NWSTEPS);
  hipMalloc(&out, (size_t)64 * 96 * 4096);
  hipMemset(W, 0, (size_t)WSTEP * NWSTEPS);
  bool cold = false;
  auto per_step = [&](const char* name, auto launch) {
    auto l2 = [&](int s) {
      if (cold) hipLaunchKernelGGL(rewrite, dim3(256), dim3(256), 0, 0, (u32x4*)W, WSTEP * NWSTEPS / 16, 0u);
      launch(s);
    };
    const float t24 = timeit([&] { l2(24); }), t96 = timeit([&] { l2(96); });
    printf("%-24s %s %7.1f ns/step   (24-step launch %8.1f ns)\n", name, cold ? "cold" : "warm", (t96 - t24) / 72.f, t24);
  };
  hipFuncSetAttribute((const void*)kB<2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 2 * WSTEP);
  hipFuncSetAttribute((const void*)kB<4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 2 * WSTEP);
  hipFuncSetAttribute((const void*)kB<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 2 * WSTEP);
  hipFuncSetAttribute((const void*)kB<4, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 2 * WSTEP);
  hipFuncSetAttribute((const void*)kB<8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 2 * WSTEP);
  const int sh = 8192 + 2 * WSTEP;
  unsigned* err;
  hipMalloc(&err, 4);
  hipMemset(err, 0, 4);
  hipFuncSetAttribute((const void*)kC<2, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 2 * WSTEP + 64);
  hipFuncSetAttribute((const void*)kC<3, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 3 * WSTEP + 64);
  hipFuncSetAttribute((const void*)kC<3, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 3 * WSTEP + 64);
  hipFuncSetAttribute((const void*)kC<3, 0, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 3 * WSTEP + 64);
  hipFuncSetAttribute((const void*)kC<3, 0, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 3 * WSTEP + 64);
  hipFuncSetAttribute((const void*)kC<3, 2, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 3 * WSTEP + 64);
  if (argc > 1 && argv[1][0] == 'E') {  // B from a resident LDS image vs streamed
    hipFuncSetAttribute((const void*)kE<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 32768);
    hipFuncSetAttribute((const void*)kE<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 32768);
    for (int rep = 0; rep < 2; ++rep) {
      per_step("A LA=2 (the chain's form)", [&](int s) { hipLaunchKernelGGL((kA<0, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
      per_step("E B from LDS (tr reads)", [&](int s) { hipLaunchKernelGGL((kE<0>), dim3(64), dim3(512), 8192 + 32768, 0, W, out, s); });
      per_step("A LA=2 no loads", [&](int s) { hipLaunchKernelGGL((kA<1, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
      per_step("A LA=2 no stores", [&](int s) { hipLaunchKernelGGL((kA<2, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
      per_step("E B from LDS, no stores", [&](int s) { hipLaunchKernelGGL((kE<2>), dim3(64), dim3(512), 8192 + 32768, 0, W, out, s); });
    }
    return 0;
  }
  if (only_d) {
    unsigned* ctr;
    __bf16* xch;
    hipMalloc(&ctr, 64 * 64 * 4);
    hipMalloc(&xch, (size_t)64 * 2 * 4096);
    auto d = [&](auto kern, int K) {
      return [=](int s) {
        hipMemsetAsync(ctr, 0, 64 * 64 * 4, 0);
        hipLaunchKernelGGL(kern, dim3(64 * K), dim3(512), 8192, 0, W, out, s, ctr, xch, err);
      };
    };
    per_step("A LA=2 (the chain's form)", [&](int s) { hipMemsetAsync(ctr, 0, 64 * 64 * 4, 0);
                                              hipLaunchKernelGGL((kA<0, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("D K=1 exchange", d(kD<1, 0>, 1));
    per_step("D K=2 exchange", d(kD<2, 0>, 2));
    per_step("D K=4 exchange", d(kD<4, 0>, 4));
    per_step("D K=2 exchange no st", d(kD<2, 2>, 2));
    per_step("D K=4 exchange no st", d(kD<4, 2>, 4));
    per_step("D K=2 no exchange", d(kD<2, 4>, 2));
    per_step("D K=4 no exchange", d(kD<4, 4>, 4));
    per_step("D K=1 no exchange", d(kD<1, 4>, 1));
    unsigned herr = 0;
    hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
    printf("spin time-outs: %u\n", herr);
    return 0;
  }
  for (int c = 0; c < 1; ++c) {
    cold = c == 1;
    per_step("C ring NS=2", [&](int s) { hipLaunchKernelGGL((kC<2, 0>), dim3(64), dim3(576), 8192 + 2 * WSTEP + 64, 0, W, out, s, err); });
    per_step("C ring NS=3", [&](int s) { hipLaunchKernelGGL((kC<3, 0>), dim3(64), dim3(576), 8192 + 3 * WSTEP + 64, 0, W, out, s, err); });
    per_step("C ring NS=3 no stores", [&](int s) { hipLaunchKernelGGL((kC<3, 2>), dim3(64), dim3(576), 8192 + 3 * WSTEP + 64, 0, W, out, s, err); });
    per_step("C ring NS=3 L=4", [&](int s) { hipLaunchKernelGGL((kC<3, 0, 4>), dim3(64), dim3(768), 8192 + 3 * WSTEP + 64, 0, W, out, s, err); });
    per_step("C ring NS=3 L=8", [&](int s) { hipLaunchKernelGGL((kC<3, 0, 8>), dim3(64), dim3(1024), 8192 + 3 * WSTEP + 64, 0, W, out, s, err); });
    per_step("C ring NS=3 L=8 no st", [&](int s) { hipLaunchKernelGGL((kC<3, 2, 8>), dim3(64), dim3(1024), 8192 + 3 * WSTEP + 64, 0, W, out, s, err); });
    per_step("A LA=1", [&](int s) { hipLaunchKernelGGL((kA<0, 2>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=2", [&](int s) { hipLaunchKernelGGL((kA<0, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=3", [&](int s) { hipLaunchKernelGGL((kA<0, 4>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=5", [&](int s) { hipLaunchKernelGGL((kA<0, 6>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=2 issue first", [&](int s) { hipLaunchKernelGGL((kA<4, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=3 issue first", [&](int s) { hipLaunchKernelGGL((kA<4, 4>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=2 16B stores, 4 waves", [&](int s) { hipLaunchKernelGGL((kA<16, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=2 staggered", [&](int s) { hipLaunchKernelGGL((kA<8, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=3 staggered", [&](int s) { hipLaunchKernelGGL((kA<8, 4>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=2 issue first no st", [&](int s) { hipLaunchKernelGGL((kA<6, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=2 no stores", [&](int s) { hipLaunchKernelGGL((kA<2, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A LA=2 no loads", [&](int s) { hipLaunchKernelGGL((kA<1, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    per_step("A no loads no stores", [&](int s) { hipLaunchKernelGGL((kA<3, 3>), dim3(64), dim3(512), 8192, 0, W, out, s); });
    if (c == 1 || c == 0) continue;
    per_step("B L=2 LA=1", [&](int s) { hipLaunchKernelGGL((kB<2, 1>), dim3(64), dim3(640), sh, 0, W, out, s); });
    per_step("B L=4 LA=1", [&](int s) { hipLaunchKernelGGL((kB<4, 1>), dim3(64), dim3(768), sh, 0, W, out, s); });
    per_step("B L=4 LA=2", [&](int s) { hipLaunchKernelGGL((kB<4, 2>), dim3(64), dim3(768), sh, 0, W, out, s); });
    per_step("B L=4 LA=3", [&](int s) { hipLaunchKernelGGL((kB<4, 3>), dim3(64), dim3(768), sh, 0, W, out, s); });
    per_step("B L=8 LA=2", [&](int s) { hipLaunchKernelGGL((kB<8, 2>), dim3(64), dim3(1024), sh, 0, W, out, s); });
  }
  unsigned herr = 0;
  hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
  printf("spin time-outs: %u\n", herr);
  return 0;
}
