// Microbenchmark (GPU box): the row chain's weight-stream access pattern in isolation.
// 64 workgroups x 8 waves; every step each wave loads one 4 x 16-B-per-lane block (its 16 rows x
// 128 K of a shared 32 KB bf16 matrix, the same lines for all workgroups), double-buffered one
// step ahead, then optionally does ALU filler and 4 scattered 2-B stores, then s_barrier.
// Prints ns per step for each mode.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))

template <int MODE>  // bit0: stores, bit1: filler ALU, bit2: no loads, bit3: MFMA on the block
__global__ __launch_bounds__(512) void k(const __bf16* W, __bf16* out, int steps, int filler, float* sink) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, kq = (lane >> 4) * 8;
  const __bf16* w0 = (MODE & 16) ? W + ((size_t)wave * 4 * 64 + lane) * 8 : W + (size_t)(wave * 16 + r16) * 128 + kq;
  const int ustride = (MODE & 16) ? 64 * 8 : 32;  // fragment order: chunk u of this wave = 1 KB contiguous
  bf16x8 pre[4], cur[4];
  auto load = [&](bf16x8* b) {
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = (MODE & 4) ? bf16x8{} : *(const G bf16x8*)(w0 + u * ustride);
  };
  load(pre);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float x = (float)lane;
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = pre[u];
    load(pre);
    if (MODE & 8) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[u], cur[u], acc, 0, 0, 0);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[0] += (float)cur[u][0] + (float)cur[u][7];
    }
    if (MODE & 2)
      for (int i = 0; i < filler; ++i) x = x * 1.0001f + 0.5f;
    if (MODE & 1) {
      __bf16* o = out + (size_t)(wave * 16 + (lane >> 4) * 4) * 1024 + blockIdx.x * 16 + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) *(G __bf16*)(o + i * 1024) = (__bf16)(acc[i] + x);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] + x == 12345.f) sink[0] = 1.f;
}

// explicit A/B double buffer: the loop is unrolled by two so neither slot is ever copied
template <int MODE>
__global__ __launch_bounds__(512) void kab(const __bf16* W, __bf16* out, int steps, int filler, float* sink) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, kq = (lane >> 4) * 8;
  const __bf16* w0 = W + (size_t)(wave * 16 + r16) * 128 + kq;
  bf16x8 A[4], B[4];
  auto load = [&](bf16x8* b) {
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = *(const G bf16x8*)(w0 + u * 32);
  };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float x = (float)lane;
  auto body = [&](bf16x8* c, bf16x8* n) {
    load(n);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c[u], c[u], acc, 0, 0, 0);
    if (MODE & 2)
      for (int i = 0; i < filler; ++i) x = x * 1.0001f + 0.5f;
    if (MODE & 1) {
      __bf16* o = out + (size_t)(wave * 16 + (lane >> 4) * 4) * 1024 + blockIdx.x * 16 + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) *(G __bf16*)(o + i * 1024) = (__bf16)(acc[i] + x);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  load(A);
  for (int s = 0; s < steps; s += 2) {
    body(A, B);
    body(B, A);
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] + x == 12345.f) sink[0] = 1.f;
}

template <int MODE, bool AB = false>
float run(const __bf16* W, __bf16* out, float* sink, int steps, int filler) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  auto kern = AB ? kab<MODE> : k<MODE>;
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(64), dim3(512), 0, 0, W, out, steps, filler, sink);
  hipEventRecord(a);
  const int reps = 20;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(64), dim3(512), 0, 0, W, out, steps, filler, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 1e6f / reps;  // ns per launch
}

int main() {
  __bf16 *W, *out; float* sink;
  hipMalloc(&W, 128 * 128 * 2); hipMalloc(&out, 128 * 1024 * 2 * 2); hipMalloc(&sink, 4);
  hipMemset(W, 0, 128 * 128 * 2);
  auto per_step = [&](auto f, const char* name, int filler) {
    const float t40 = f(40, filler), t80 = f(80, filler);
    printf("%-34s filler=%4d  %7.1f ns/step  (launch 40 steps %8.1f ns)\n", name, filler, (t80 - t40) / 40.f, t40);
  };
  per_step([&](int s, int fl) { return run<16 + 8>(W, out, sink, s, fl); }, "FRAG loads + MFMA", 0);
  per_step([&](int s, int fl) { return run<16 + 8 + 1>(W, out, sink, s, fl); }, "FRAG loads + MFMA + stores", 0);
  per_step([&](int s, int fl) { return run<16 + 2>(W, out, sink, s, fl); }, "FRAG loads + filler", 50);
  per_step([&](int s, int fl) { return run<0, true>(W, out, sink, s, fl); }, "AB loads + MFMA", 0);
  per_step([&](int s, int fl) { return run<1, true>(W, out, sink, s, fl); }, "AB loads + MFMA + stores", 0);
  for (int fl : {50, 200}) {
    per_step([&](int s, int f2) { return run<2, true>(W, out, sink, s, f2); }, "AB loads + filler", fl);
    per_step([&](int s, int f2) { return run<3, true>(W, out, sink, s, f2); }, "AB loads + filler + stores", fl);
  }
  per_step([&](int s, int fl) { return run<4>(W, out, sink, s, fl); }, "no loads", 0);
  per_step([&](int s, int fl) { return run<0>(W, out, sink, s, fl); }, "loads", 0);
  per_step([&](int s, int fl) { return run<8>(W, out, sink, s, fl); }, "loads + 4 MFMA", 0);
  per_step([&](int s, int fl) { return run<12>(W, out, sink, s, fl); }, "no loads + 4 MFMA", 0);
  per_step([&](int s, int fl) { return run<1>(W, out, sink, s, fl); }, "loads + stores", 0);
  per_step([&](int s, int fl) { return run<5>(W, out, sink, s, fl); }, "no loads + stores", 0);
  for (int fl : {50, 200, 800}) {
    per_step([&](int s, int f2) { return run<2>(W, out, sink, s, f2); }, "loads + filler", fl);
    per_step([&](int s, int f2) { return run<6>(W, out, sink, s, f2); }, "no loads + filler", fl);
    per_step([&](int s, int f2) { return run<3>(W, out, sink, s, f2); }, "loads + filler + stores", fl);
  }
  return 0;
}
