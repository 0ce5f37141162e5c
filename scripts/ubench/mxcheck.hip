// Probe: v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 A/B, unit E8M0 scales) on two consecutive 16-B
// K-pair fragments per lane == four v_mfma_f32_16x16x32_fp8_fp8 over the same bytes (the pair
// layout of cvae_widechain.h: 8 B per 32-wide K chunk per lane).  Prints the max |difference|.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void probe(const v8i* a, const v8i* b, f4* c1, f4* c2) {
  const int l = threadIdx.x;
  const v8i A = a[l], B = b[l];
  f4 x = {0.f, 0.f, 0.f, 0.f}, y = {0.f, 0.f, 0.f, 0.f};
  x = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, x, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  for (int h = 0; h < 4; ++h) {
    const long av = (long)(unsigned)A[2 * h] | ((long)(unsigned)A[2 * h + 1] << 32);
    const long bv = (long)(unsigned)B[2 * h] | ((long)(unsigned)B[2 * h + 1] << 32);
    y = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av, bv, y, 0, 0, 0);
  }
  c1[l] = x;
  c2[l] = y;
}
int main() {
  const int N = 64;
  v8i ha[N], hb[N];
  srand(7);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < 8; ++j) {
      unsigned wa = 0, wb = 0;
      for (int k = 0; k < 4; ++k) {  // e4m3 bytes with exponent field < 15 (finite, no NaN)
        wa |= (unsigned)((rand() & 0x87) | ((rand() % 14) << 3)) << (8 * k);
        wb |= (unsigned)((rand() & 0x87) | ((rand() % 14) << 3)) << (8 * k);
      }
      ha[i][j] = (int)wa;
      hb[i][j] = (int)wb;
    }
  v8i *da, *db;
  f4 *d1, *d2;
  hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb);
  hipMalloc(&d1, N * sizeof(f4)); hipMalloc(&d2, N * sizeof(f4));
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, d1, d2);
  f4 r1[N], r2[N];
  hipMemcpy(r1, d1, sizeof r1, hipMemcpyDeviceToHost);
  hipMemcpy(r2, d2, sizeof r2, hipMemcpyDeviceToHost);
  double md = 0, mx = 0;
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < 4; ++k) {
      md = fmax(md, fabs((double)r1[i][k] - (double)r2[i][k]));
      mx = fmax(mx, fabs((double)r2[i][k]));
    }
  printf("scaled 16x16x128 vs 4 x 16x16x32 fp8: max |diff| %.6g, max |value| %.6g\n", md, mx);
  return md <= 1e-4 * mx ? 0 : 1;
}
