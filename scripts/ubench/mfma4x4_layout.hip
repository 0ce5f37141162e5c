// Probe (GPU box) for the fp32 chain's 4-row form (cvae_f32chain.h):
//  1. the operand and result lanes of v_mfma_f32_4x4x1_16b_f32 as mm4<4> uses them: A lane l = row
//     l % 4 of block l / 4, B lane l = column l % 4 of block l / 4, result lane l element i =
//     D[block l / 4][row i][column l % 4];
//  2. kred's row-swap sums (v_permlane16_swap / v_permlane32_swap of a value with itself) equal the
//     ds_bpermute butterfly (v + v^16, then + v^32) bit for bit on random floats.
// Prints "layout ok" / "kred ok" or the first mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(float* out) {
  const int l = threadIdx.x;
  const float a = 1.f + l, b = 100.f + 3 * l;
  const f32x4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[l * 4 + i] = d[i];
}

__global__ void kr(const float* in, float* swp, float* shf) {
  const int l = threadIdx.x + 64 * blockIdx.x;
  auto u = [](float f) { return __builtin_bit_cast(unsigned, f); };
  auto f = [](unsigned x) { return __builtin_bit_cast(float, x); };
  float v = in[l];
  const auto r = __builtin_amdgcn_permlane16_swap(u(v), u(v), false, false);
  v = f(r[0]) + f(r[1]);
  const auto s = __builtin_amdgcn_permlane32_swap(u(v), u(v), false, false);
  swp[l] = f(s[0]) + f(s[1]);
  float w = in[l];
  w += __shfl_xor(w, 16);
  w += __shfl_xor(w, 32);
  shf[l] = w;
}

int main() {
  float* o;
  (void)hipMalloc(&o, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o);
  float h[256];
  (void)hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int blk = l / 4, j = l % 4;
      const float want = (1.f + (4 * blk + i)) * (100.f + 3 * (4 * blk + j));
      if (h[l * 4 + i] != want) {
        printf("mismatch lane %d elem %d: %g want %g\n", l, i, h[l * 4 + i], want);
        return 1;
      }
    }
  printf("layout ok\n");
  const int N = 64 * 1024;
  float *in, *a, *b;
  (void)hipMalloc(&in, N * 4);
  (void)hipMalloc(&a, N * 4);
  (void)hipMalloc(&b, N * 4);
  float* hi = (float*)malloc(N * 4);
  srand(1);
  for (int i = 0; i < N; ++i) hi[i] = ((float)rand() / RAND_MAX - 0.5f) * (float)(1 << (rand() % 20));
  (void)hipMemcpy(in, hi, N * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(kr, dim3(N / 64), dim3(64), 0, 0, in, a, b);
  float* ha = (float*)malloc(N * 4);
  float* hb = (float*)malloc(N * 4);
  (void)hipMemcpy(ha, a, N * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hb, b, N * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < N; ++i)
    if (__builtin_bit_cast(unsigned, ha[i]) != __builtin_bit_cast(unsigned, hb[i])) {
      printf("kred mismatch at %d: swap %a butterfly %a\n", i, ha[i], hb[i]);
      return 1;
    }
  printf("kred ok\n");
  return 0;
}
