// Probe (GPU box): gfx950 bf16 -> e4m3 conversions.  v_cvt_scalef32_pk_fp8_bf16 (2 bf16 straight
// to 2 e4m3, scale 1) against v_cvt_pk_fp8_f32 on clamped floats, over every bf16 bit pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned short* in, unsigned char* a, unsigned char* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  unsigned short u0 = in[2 * i], u1 = in[2 * i + 1];
  bf16x2 v;
  v[0] = __builtin_bit_cast(__bf16, u0);
  v[1] = __builtin_bit_cast(__bf16, u1);
  i16x2 old = {0, 0};
  i16x2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(old, v, 1.0f, false);
  unsigned w = __builtin_bit_cast(unsigned, r);
  a[2 * i] = w & 0xFF; a[2 * i + 1] = (w >> 8) & 0xFF;
  float f0 = fminf(fmaxf((float)v[0], -448.f), 448.f), f1 = fminf(fmaxf((float)v[1], -448.f), 448.f);
  int w2 = __builtin_amdgcn_cvt_pk_fp8_f32(f0, f1, 0, false);
  b[2 * i] = w2 & 0xFF; b[2 * i + 1] = (w2 >> 8) & 0xFF;
}
int main() {
  const int n = 65536;
  unsigned short h[n];
  for (int i = 0; i < n; ++i) h[i] = (unsigned short)i;
  unsigned short* d; unsigned char *a, *b;
  hipMalloc(&d, n * 2); hipMalloc(&a, n); hipMalloc(&b, n);
  hipMemcpy(d, h, n * 2, hipMemcpyHostToDevice);
  k<<<n / 2 / 256, 256>>>(d, a, b, n);
  static unsigned char ha[n], hb[n];
  hipMemcpy(ha, a, n, hipMemcpyDeviceToHost); hipMemcpy(hb, b, n, hipMemcpyDeviceToHost);
  int diff = 0, diff_finite = 0;
  for (int i = 0; i < n; ++i) {
    const bool nan = (h[i] & 0x7F80) == 0x7F80;
    if (ha[i] != hb[i]) { ++diff; if (!nan) { ++diff_finite; if (diff_finite < 12) printf("bf16 %04x: scalef32 %02x clamp+f32 %02x\n", h[i], ha[i], hb[i]); } }
  }
  // spot values: 500, -1e4, 1.0625, 2^-10
  printf("diff %d (finite inputs %d)\n", diff, diff_finite);
  printf("500 -> %02x / %02x ; 1.0 -> %02x\n", ha[0x43FA], hb[0x43FA], ha[0x3F80]);
  return 0;
}
