// Microbenchmark (GPU box): the fp32 chain's 128 × 128 step at the reference's own batch (B = 32),
// priced in two tilings (the cfg1 lever).  Every step reads a fresh 64-KB block of fp32
// weights (the same lines in every workgroup) and writes its activations back to LDS for the next
// step and to global memory (as the chain's arena copy).
//   T16: the current form — 2 workgroups × 16 rows; wave w owns n-tile w (16 features) over all
//        K = 128: 32 × v_mfma_f32_16x16x4_f32 per wave per step (0.85 us of MFMA issue per step at
//        2 waves per SIMD).
//   T4:  4-row tiles — 8 workgroups × 4 rows; v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4 × 4 × 1: 64
//        features × 4 rows per instruction); wave w takes feature half w & 1 and K quarter w >> 1 (32
//        MFMAs per wave per step, 1/4 of the MFMA issue), the quarters' partial sums meet in LDS in a
//        fixed order, one more barrier per step.
// Prints ns per step (difference of two step counts: launch overhead cancels).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))

constexpr int WSTEP = 64 * 1024;  // fp32 weight bytes per step per workgroup (128 × 128)
constexpr int NWSTEPS = 48;       // distinct weight blocks (3 MB)

__device__ __forceinline__ void lbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// T16: 16 rows, LDS image [chunk c (16 features)][lane (r, q)][4]: lane (r, q) = row r's features
// 16c + 4q .. +3 (the f32 chain's fragment image); the swapped MFMA acc = W·Xᵀ leaves n-tile t's
// outputs in exactly that slot order
template <int NB>
__global__ __launch_bounds__(512) void kT16(const float* W, float* out, int nstep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto img = [&](int i) { return (float*)(smem + (i & 1) * 8192); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 512) ((f32x4*)smem)[tid] = f32x4{0.01f, 0.01f, 0.01f, 0.01f};
  f32x4 w[NB][8];  // this wave's n-tile: 8 chunks of 16 K (4 k per MFMA × 4 MFMAs per 1-KB fragment)
  auto wl = [&](f32x4* wr, int s) {
    const float* p = W + (size_t)(s % NWSTEPS) * (WSTEP / 4) + ((size_t)wave * 8 * 64 + lane) * 4;
#pragma unroll
    for (int c = 0; c < 8; ++c) wr[c] = *(const G f32x4*)(p + c * 256);
  };
#pragma unroll
  for (int b = 0; b < NB - 1; ++b) wl(w[b], b);
  lbar();
  for (int s0 = 0; s0 < nstep; s0 += NB) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int s = s0 + b;
      const float* in = img(s);
      float* o = img(s + 1);
      wl(w[(b + NB - 1) % NB], s + NB - 1);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const f32x4 x = *(const f32x4*)(in + (c * 64 + lane) * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w[b][c][e], x[e], acc, 0, 0, 0);
      }
      f32x4 h;
#pragma unroll
      for (int i = 0; i < 4; ++i) h[i] = fmaxf(acc[i] * 0.01f, 0.f);
      *(f32x4*)(o + (wave * 64 + lane) * 4) = h;
      *(G f32x4*)(out + (((size_t)blockIdx.x * nstep + s) * 512 + wave * 64 + lane) * 4) = h;
      lbar();
    }
  }
}

// T4: 4 rows, LDS image X[row][128] fp32 (lane (b, j) reads row j: 4 distinct addresses per wave,
// broadcast); partials [quarter][half][lane] f32x4
template <int NB>
__global__ __launch_bounds__(512) void kT4(const float* W, float* out, int nstep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto img = [&](int i) { return (float*)(smem + (i & 1) * 2048); };
  float* const part = (float*)(smem + 4096);  // 4 quarters × 2 halves × 64 lanes × 16 B = 8 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = wave & 1, kq = wave >> 1;
  const int j = lane & 3;  // the row this lane supplies as the B operand (and receives outputs of)
  if (tid < 256) ((f32x4*)smem)[tid] = f32x4{0.01f, 0.01f, 0.01f, 0.01f};
  f32x4 w[NB][8];  // feature 64h + lane, k = 32kq + 4c .. +3
  auto wl = [&](f32x4* wr, int s) {
    const float* p = W + (size_t)(s % NWSTEPS) * (WSTEP / 4) + ((size_t)(h * 4 + kq) * 8 * 64 + lane) * 4;
#pragma unroll
    for (int c = 0; c < 8; ++c) wr[c] = *(const G f32x4*)(p + c * 256);
  };
#pragma unroll
  for (int b = 0; b < NB - 1; ++b) wl(w[b], b);
  lbar();
  for (int s0 = 0; s0 < nstep; s0 += NB) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int s = s0 + b;
      const float* in = img(s);
      float* o = img(s + 1);
      wl(w[(b + NB - 1) % NB], s + NB - 1);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const f32x4 x = *(const f32x4*)(in + j * 128 + kq * 32 + 4 * c);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(w[b][c][e], x[e], acc, 0, 0, 0);
      }
      *(f32x4*)(part + ((kq * 2 + h) * 64 + lane) * 4) = acc;
      lbar();
      // output (row r, feature n) of thread t: the 4 quarters' partials, summed in quarter order
      const int n = tid & 127, r = tid >> 7;
      const int hh = n >> 6, l = ((n & 63) >> 2) * 4 + r, i = n & 3;
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) v += part[((q * 2 + hh) * 64 + l) * 4 + i];
      v = fmaxf(v * 0.01f, 0.f);
      o[r * 128 + n] = v;
      out[((size_t)blockIdx.x * nstep + s) * 512 + tid] = v;
      lbar();
    }
  }
}

template <class F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 20; ++r) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  return best * 1e6f;  // ns
}

int main() {
  float *W, *out;
  hipMalloc(&W, (size_t)WSTEP * NWSTEPS);
  hipMalloc(&out, (size_t)8 * 96 * 512 * 4);
  hipMemset(W, 0, (size_t)WSTEP * NWSTEPS);
  auto per_step = [&](const char* name, auto launch) {
    const float t24 = timeit([&] { launch(24); }), t96 = timeit([&] { launch(96); });
    printf("%-40s %7.1f ns/step   (24-step launch %8.1f ns)\n", name, (t96 - t24) / 72.f, t24);
  };
  for (int rep = 0; rep < 2; ++rep) {
    per_step("T16 2 x 16 rows (the chain's form), LA=1", [&](int s) { hipLaunchKernelGGL((kT16<2>), dim3(2), dim3(512), 16384, 0, W, out, s); });
    per_step("T16 2 x 16 rows, LA=2", [&](int s) { hipLaunchKernelGGL((kT16<3>), dim3(2), dim3(512), 16384, 0, W, out, s); });
    per_step("T4 8 x 4 rows, LA=1", [&](int s) { hipLaunchKernelGGL((kT4<2>), dim3(8), dim3(512), 4096 + 8192, 0, W, out, s); });
    per_step("T4 8 x 4 rows, LA=2", [&](int s) { hipLaunchKernelGGL((kT4<3>), dim3(8), dim3(512), 4096 + 8192, 0, W, out, s); });
  }
  return 0;
}
