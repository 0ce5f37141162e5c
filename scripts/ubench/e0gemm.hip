// The encoder-L1 GEMM in isolation (Training_VAE.py:141-151: the first nn.Linear of `encoder`, I = 600
// inputs -> H = 128 features, then ReLU) at large batch: what MFMA utilisation this GEMM can reach
// on its own (BASELINE.md's ">= 50 % MFMA utilisation on the encoder GEMM"), measured beside its
// rooflines.  Not the product path (the training step runs this GEMM inside the row chain).
//
//   Y = ReLU(X · Wᵀ + b):  X [M][608] bf16 row-major (K zero-padded to 608, streamed from HBM once),
//   W [128][608] bf16 in MFMA fragment order, staged once per workgroup into LDS (152 KB),
//   Y bf16, feature-major 16-row tiles ([tile][128][16], 8-B stores).
//
// Per row: 2·608·128 FLOP against 1216 B of X + 256 B of Y → 105.7 FLOP/B, below the MI355X bf16
// ridge (2.5 PFLOP/s / 8 TB/s = 312 FLOP/B): HBM bounds this GEMM at ~0.85 PFLOP/s = 34 % of the
// dense bf16 MFMA peak at ANY batch (41 % if Y were not written).
//
// One workgroup per CU (the LDS copy of W), 8 waves; a wave owns 64 rows (4 MFMA row tiles) per
// iteration: per 32-wide K chunk it loads its 4 A fragments (16 B per lane, 3 chunks ahead), reads
// the 8 W fragments of the chunk from LDS once and issues 32 v_mfma_f32_16x16x32_bf16 (8 n-tiles x
// 4 row tiles: LDS traffic per MFMA a quarter of one-row-tile-per-wave).
//
// Variants: -DE0_RT (row tiles per wave), -DE0_NWV (waves per workgroup), -DE0_PF (chunks prefetched).
// usage: e0gemm [M] [reps]   → prints ms/launch, TFLOP/s, HBM GB/s, MFMA fraction of 2.5 PF
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifndef E0_RT
#define E0_RT 4
#endif
#ifndef E0_NWV
#define E0_NWV 8
#endif
#ifndef E0_PF
#define E0_PF 3
#endif
constexpr int K = 608, KC = K / 32, N = 128, NTI = N / 16, RT = E0_RT, NWV = E0_NWV, PF = E0_PF;
constexpr int W_BYTES = N * K * 2;  // 155,648 B

__global__ __launch_bounds__(64 * NWV) void e0_gemm(const __bf16* __restrict__ X, const u32x4* __restrict__ Wfrag,
                                               const float* __restrict__ bias, __bf16* __restrict__ Y, int M) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // W: 152 KB of fragments into LDS (whole 16-B vectors)
  for (int i = tid; i < W_BYTES / 16; i += 64 * NWV) ((u32x4*)smem)[i] = Wfrag[i];
  __syncthreads();
  const int r = lane & 15, q = lane >> 4;
  float bq[NTI];
#pragma unroll
  for (int t = 0; t < NTI; ++t) bq[t] = bias[16 * t + r];
  const int tiles = M / (16 * RT);  // 64-row groups
  for (int g = blockIdx.x * NWV + wave; g < tiles; g += gridDim.x * NWV) {
    const __bf16* xg = X + (size_t)g * (16 * RT) * K + (size_t)r * K + 8 * q;
    bf16x8 a[PF][RT];
#pragma unroll
    for (int c = 0; c < PF; ++c)
#pragma unroll
      for (int u = 0; u < RT; ++u) a[c][u] = *(const bf16x8*)(xg + (size_t)u * 16 * K + 32 * c);
    f32x4 acc[RT][NTI];
#pragma unroll
    for (int u = 0; u < RT; ++u)
#pragma unroll
      for (int t = 0; t < NTI; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      bf16x8 cur[RT];
#pragma unroll
      for (int u = 0; u < RT; ++u) cur[u] = a[c % PF][u];
      if (c + PF < KC) {
#pragma unroll
        for (int u = 0; u < RT; ++u) a[c % PF][u] = *(const bf16x8*)(xg + (size_t)u * 16 * K + 32 * (c + PF));
      }
#pragma unroll
      for (int t = 0; t < NTI; ++t) {
        const bf16x8 w = *(const bf16x8*)(smem + ((size_t)(t * KC + c) * 64 + lane) * 16);
#pragma unroll
        for (int u = 0; u < RT; ++u) acc[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[u], w, acc[u][t], 0, 0, 0);
      }
      // keep each chunk's prefetch in its own iteration: left free, the scheduler hoists the loads of
      // all 19 chunks to the top (19 x 4 fragments live: spills)
      __builtin_amdgcn_sched_barrier(0);
    }
    // bias + ReLU; lane holds rows 4q..4q+3 of tile u, feature 16t + r: 8-B stores, feature-major tiles
#pragma unroll
    for (int u = 0; u < RT; ++u) {
      __bf16* yt = Y + (size_t)(g * RT + u) * N * 16;
#pragma unroll
      for (int t = 0; t < NTI; ++t) {
        bf16x4 h;
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = (__bf16)fmaxf(acc[u][t][i] + bq[t], 0.f);
        *(bf16x4*)(yt + (16 * t + r) * 16 + 4 * q) = h;
      }
    }
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : (1 << 18);
  const int reps = argc > 2 ? atoi(argv[2]) : 50;
  if (M % (16 * RT)) { fprintf(stderr, "M must be a multiple of %d\n", 16 * RT); return 2; }
  std::vector<__bf16> hx((size_t)M * K), hw((size_t)N * K);
  std::vector<float> hb(N);
  srand(1);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (__bf16)((i % K) < 600 ? (rand() / (float)RAND_MAX - 0.5f) : 0.f);
  for (int n = 0; n < N; ++n)
    for (int k = 0; k < K; ++k) hw[(size_t)n * K + k] = (__bf16)(k < 600 ? (rand() / (float)RAND_MAX - 0.5f) * 0.08f : 0.f);
  for (int n = 0; n < N; ++n) hb[n] = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  // fragment order of the B operand: lane (r, q) of (n-tile t, chunk c) holds W[16t + r][32c + 8q .. +7]
  // (the A fragments are loaded with the same K order, so any consistent order is exact)
  std::vector<__bf16> hf((size_t)N * K);
  for (int t = 0; t < NTI; ++t)
    for (int c = 0; c < KC; ++c)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 8; ++e)
          hf[(((size_t)(t * KC + c) * 64 + l) * 8) + e] = hw[(size_t)(16 * t + (l & 15)) * K + 32 * c + 8 * (l >> 4) + e];
  __bf16 *dx, *dy;
  u32x4* dw;
  float* db;
  hipMalloc(&dx, hx.size() * 2);
  hipMalloc(&dw, hf.size() * 2);
  hipMalloc(&db, N * 4);
  hipMalloc(&dy, (size_t)M * N * 2);
  hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dw, hf.data(), hf.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), N * 4, hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)e0_gemm, hipFuncAttributeMaxDynamicSharedMemorySize, W_BYTES);
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const dim3 grid(ncu), block(64 * NWV);
  hipLaunchKernelGGL(e0_gemm, grid, block, W_BYTES, 0, dx, dw, db, dy, M);
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "launch failed\n"); return 1; }
  // check 64 rows against a host fp32 reference of the same bf16 operands
  std::vector<__bf16> hy((size_t)M * N);
  hipMemcpy(hy.data(), dy, hy.size() * 2, hipMemcpyDeviceToHost);
  double maxerr = 0;
  for (int row = 0; row < 64; ++row) {
    const int rr = (row * 4099) % M;
    for (int n = 0; n < N; ++n) {
      double s = hb[n];
      for (int k = 0; k < K; ++k) s += (double)(float)hx[(size_t)rr * K + k] * (double)(float)hw[(size_t)n * K + k];
      s = s > 0 ? s : 0;
      const double got = (float)hy[((size_t)(rr / 16) * N + n) * 16 + rr % 16];
      maxerr = fmax(maxerr, fabs(got - s) / (fabs(s) + 1e-2));
    }
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(e0_gemm, grid, block, W_BYTES, 0, dx, dw, db, dy, M);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  const double flop = 2.0 * M * K * N, flop600 = 2.0 * M * 600 * N, bytes = (double)M * (K * 2 + N * 2);
  printf("{\"M\": %d, \"ms\": %.5f, \"tflops_k608\": %.1f, \"tflops_k600\": %.1f, \"mfma_frac_of_2500\": %.4f, "
         "\"hbm_gbs\": %.0f, \"hbm_frac_of_8000\": %.4f, \"roof_tflops\": %.1f, \"rel_err_max\": %.2e}\n",
         M, ms, flop / ms * 1e-9, flop600 / ms * 1e-9, flop / ms * 1e-9 / 2500.0, bytes / ms * 1e-6,
         bytes / ms * 1e-6 / 8000.0, flop / bytes * 8.0, maxerr);
  return maxerr < 2e-2 ? 0 : 1;
}
