// Probe (GPU box): the operand and result lanes of v_mfma_f32_4x4x1_16b_f32 as the fp32 chain's 4-row
// form uses them (cvae_f32chain.h mm4<4>): A lane l = row l % 4 of block l / 4, B lane l = column l % 4
// of block l / 4, result lane l element i = D[block l / 4][row i][column l % 4].  Prints "layout ok"
// or the first mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(float* out) {
  const int l = threadIdx.x;
  const float a = 1.f + l, b = 100.f + 3 * l;
  const f32x4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[l * 4 + i] = d[i];
}

int main() {
  float* o;
  hipMalloc(&o, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o);
  float h[256];
  hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
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
  return 0;
}
