// Probe (GPU box): the scale operand of v_cvt_scalef32_pk_fp8_bf16.  For every bf16 pattern x and
// scale exponents k, compares the instruction with scale 2^k (and 2^-k) against
// v_cvt_pk_fp8_f32(x * 2^k) (RNE, values within ±448 only) — which form multiplies, and whether it
// rounds exactly like scaling first (denormal e4m3 outputs included).  Exit 1 if neither matches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cmath>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned short* in, unsigned char* a, unsigned char* b, unsigned char* c, int n, float s) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  bf16x2 v;
  v[0] = __builtin_bit_cast(__bf16, in[2 * i]);
  v[1] = __builtin_bit_cast(__bf16, in[2 * i + 1]);
  i16x2 old = {0, 0};
  unsigned w = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(old, v, s, false));
  unsigned w3 = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(old, v, 1.f / s, false));
  a[2 * i] = w & 0xFF; a[2 * i + 1] = (w >> 8) & 0xFF;
  c[2 * i] = w3 & 0xFF; c[2 * i + 1] = (w3 >> 8) & 0xFF;
  int w2 = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[0] * s, (float)v[1] * s, 0, false);
  b[2 * i] = w2 & 0xFF; b[2 * i + 1] = (w2 >> 8) & 0xFF;
}
int main() {
  const int n = 65536;
  static unsigned short h[n];
  for (int i = 0; i < n; ++i) h[i] = (unsigned short)i;
  unsigned short* d; unsigned char *a, *b, *c;
  hipMalloc(&d, n * 2); hipMalloc(&a, n); hipMalloc(&b, n); hipMalloc(&c, n);
  hipMemcpy(d, h, n * 2, hipMemcpyHostToDevice);
  static unsigned char ha[n], hb[n], hc[n];
  int ok_mul = 1, ok_div = 1;
  for (int kk : {0, 1, 7, 20, 64, 126, -3}) {
    const float s = ldexpf(1.f, kk);
    k<<<n / 2 / 256, 256>>>(d, a, b, c, n, s);
    hipMemcpy(ha, a, n, hipMemcpyDeviceToHost); hipMemcpy(hb, b, n, hipMemcpyDeviceToHost); hipMemcpy(hc, c, n, hipMemcpyDeviceToHost);
    int dm = 0, dd = 0, cnt = 0;
    for (int i = 0; i < n; ++i) {
      unsigned u = (unsigned)h[i] << 16; float x; memcpy(&x, &u, 4);
      if (!(fabsf(x * s) <= 448.f)) continue;  // finite and in range
      ++cnt;
      if (ha[i] != hb[i]) { if (dm < 4) printf("k=%d x=%04x: scale 2^k %02x, x*2^k %02x\n", kk, h[i], ha[i], hb[i]); ++dm; }
      if (hc[i] != hb[i]) ++dd;
    }
    printf("k=%4d: %d in-range inputs; scale=2^k differs %d, scale=2^-k differs %d\n", kk, cnt, dm, dd);
    if (dm) ok_mul = 0;
    if (dd) ok_div = 0;
  }
  printf(ok_mul ? "the instruction multiplies by its scale (bit-equal to x*2^k then RNE)\n"
                : ok_div ? "the instruction divides by its scale (bit-equal to x/2^k then RNE)\n"
                         : "neither form is bit-equal\n");
  return ok_mul || ok_div ? 0 : 1;
}
