// Microbenchmark (GPU box): per-CU streaming rates the row chain depends on, 64 workgroups (one
// per CU) as in the real launch.  Each workgroup streams TOT bytes of a shared read-only buffer
// (the weights: every workgroup reads the same lines) or writes its own 512-B-run output.
//   regld   : 8 waves, 16-B-per-lane global loads into registers, PF instructions in flight per wave
//   glds<L> : L loader waves, global_load_lds_dwordx4 into a 64-KB LDS ring, 16 in flight per wave
//   st8/st16: 8 waves, 8-B / 16-B-per-lane stores (512 B / 1 KB contiguous per wave instruction)
// Prints us per launch and GB/s per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#define G __attribute__((address_space(1)))
#define LDSP __attribute__((address_space(3)))

template <int PF>
__global__ __launch_bounds__(512) void regld(const char* W, int tot, unsigned* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per_wave = tot / 8;
  const char* p = W + (size_t)wave * per_wave + lane * 16;
  u32x4 acc = {0, 0, 0, 0};
  for (int off = 0; off < per_wave; off += PF * 1024) {
    u32x4 v[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) v[u] = *(const G u32x4*)(p + off + u * 1024);
#pragma unroll
    for (int u = 0; u < PF; ++u) acc ^= v[u];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;
}

// the same stream with workgroup b starting ROT·b bytes further into its slice (wrapping): the 64
// workgroups no longer request the same lines at the same moment (hot L2 channels); PRIV: each
// workgroup streams its own copy of the buffer (no sharing at all)
template <int PF, bool PRIV>
__global__ __launch_bounds__(512) void regld_rot(const char* W, int tot, int rot, unsigned* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per_wave = tot / 8;
  const char* p = W + (PRIV ? (size_t)blockIdx.x * tot : 0) + (size_t)wave * per_wave + lane * 16;
  const int r0 = (int)(((long)blockIdx.x * rot) % per_wave) & ~1023;
  u32x4 acc = {0, 0, 0, 0};
  for (int off = 0; off < per_wave; off += PF * 1024) {
    u32x4 v[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      int o = off + u * 1024 + r0;
      o = o >= per_wave ? o - per_wave : o;
      v[u] = *(const G u32x4*)(p + o);
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) acc ^= v[u];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;
}

template <int L>
__global__ __launch_bounds__(64 * L) void glds(const char* W, int tot, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) char ring[65536];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per_wave = tot / L;
  const char* p = W + (size_t)wave * per_wave + lane * 16;
  LDSP char* r = (LDSP char*)ring + wave * (65536 / L);
  const int slots = 65536 / L / 1024;
  int s = 0;
  for (int off = 0; off < per_wave; off += 1024) {
    __builtin_amdgcn_global_load_lds((const G void*)(p + off), (LDSP void*)(r + s * 1024), 16, 0, 0);
    s = s + 1 == slots ? 0 : s + 1;
    if ((off >> 10) % 16 == 15) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ring[threadIdx.x * 16] == 123) sink[0] = 1;
}

template <int BYTES>
__global__ __launch_bounds__(512) void st(char* out, int tot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per_wave = tot / 8, step = 64 * BYTES;
  char* p = out + (size_t)blockIdx.x * tot + (size_t)wave * per_wave + lane * BYTES;
  for (int off = 0; off < per_wave; off += step) {
    if (BYTES == 8)
      *(G u32x2*)(p + off) = u32x2{(unsigned)off, (unsigned)lane};
    else
      *(G u32x4*)(p + off) = u32x4{(unsigned)off, (unsigned)lane, 0u, 1u};
  }
}

template <typename F>
float timeit(F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) launch();
  const int reps = 50;
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / reps;  // us per launch
}

int main() {
  const int TOT = 1 << 20, STOT = 136 * 1024;
  char *W, *out;
  unsigned* sink;
  hipMalloc(&W, TOT);
  char* WP;
  hipMalloc(&WP, (size_t)TOT * 64);
  hipMemset(WP, 1, (size_t)TOT * 64);
  hipMalloc(&out, (size_t)STOT * 64);
  hipMalloc(&sink, 4);
  hipMemset(W, 1, TOT);
  auto rep = [&](const char* name, float us, double bytes) {
    printf("%-28s %8.2f us/launch  %7.1f GB/s per CU\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  const float empty = timeit([&] { hipLaunchKernelGGL(regld<4>, dim3(64), dim3(512), 0, 0, W, 0, sink); });
  rep("empty launch", empty, 0);
  rep("regld PF=4", timeit([&] { hipLaunchKernelGGL(regld<4>, dim3(64), dim3(512), 0, 0, W, TOT, sink); }), TOT);
  rep("regld PF=8", timeit([&] { hipLaunchKernelGGL(regld<8>, dim3(64), dim3(512), 0, 0, W, TOT, sink); }), TOT);
  rep("regld PF=16", timeit([&] { hipLaunchKernelGGL(regld<16>, dim3(64), dim3(512), 0, 0, W, TOT, sink); }), TOT);
  rep("regld PF=8 x256 WG", timeit([&] { hipLaunchKernelGGL(regld<8>, dim3(256), dim3(512), 0, 0, W, TOT, sink); }), TOT);
  for (int rot : {1024, 4096, 16384, 40960})
    for (int pf : {4, 8}) {
      char name[64];
      snprintf(name, sizeof name, "regld PF=%d rot %d KB/WG", pf, rot / 1024);
      rep(name, timeit([&] {
            if (pf == 4) hipLaunchKernelGGL((regld_rot<4, false>), dim3(64), dim3(512), 0, 0, W, TOT, rot, sink);
            else hipLaunchKernelGGL((regld_rot<8, false>), dim3(64), dim3(512), 0, 0, W, TOT, rot, sink);
          }), TOT);
    }
  rep("regld PF=8 private copies", timeit([&] { hipLaunchKernelGGL((regld_rot<8, true>), dim3(64), dim3(512), 0, 0, WP, TOT, 0, sink); }), TOT);
  rep("glds L=1", timeit([&] { hipLaunchKernelGGL(glds<1>, dim3(64), dim3(64), 0, 0, W, TOT, sink); }), TOT);
  rep("glds L=2", timeit([&] { hipLaunchKernelGGL(glds<2>, dim3(64), dim3(128), 0, 0, W, TOT, sink); }), TOT);
  rep("glds L=4", timeit([&] { hipLaunchKernelGGL(glds<4>, dim3(64), dim3(256), 0, 0, W, TOT, sink); }), TOT);
  rep("glds L=8", timeit([&] { hipLaunchKernelGGL(glds<8>, dim3(64), dim3(512), 0, 0, W, TOT, sink); }), TOT);
  rep("st 8B/lane 136KB", timeit([&] { hipLaunchKernelGGL(st<8>, dim3(64), dim3(512), 0, 0, out, STOT); }), STOT);
  rep("st 16B/lane 136KB", timeit([&] { hipLaunchKernelGGL(st<16>, dim3(64), dim3(512), 0, 0, out, STOT); }), STOT);
  return 0;
}
