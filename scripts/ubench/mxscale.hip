// Probe: which E8M0 scale of v_mfma_scale_f32_16x16x128_f8f6f4 applies to which operand bytes.
// A is zero except one 8-byte quarter h of one lane La (e4m3 1.0), B is all 1.0; the output row
// La % 16 then reads 8.  For every lane Ls the A scale of Ls alone is set to 2^1 (every byte 128,
// all others 127): the output doubles iff that scale multiplies quarter (La, h).  Prints, for each
// (La, h), the lanes whose scale multiplies it.  Then the same for B (B zero except (Lb, h), A all
// 1.0), and which byte of the scale VGPR opsel 0 reads.  Measured (gfx950): quarter h of lane
// r + 16j is scaled by lane r + 16·(2·(h >> 1) + (j >> 1)) for A and B alike — the mapping
// cvae_widechain.h mx_block relies on; exit status 1 if it differs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void probe(const v8i* a, const v8i* b, const int* sa, const int* sb, f4* c) {
  const int l = threadIdx.x;
  f4 x = {0.f, 0.f, 0.f, 0.f};
  x = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], x, 0, 0, 0, sa[l], 0, sb[l]);
  c[l] = x;
}

int main() {
  const int N = 64;
  static v8i ha[N], hb[N];
  static int sa[N], sb[N];
  v8i *da, *db;
  int *dsa, *dsb;
  f4* dc;
  hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dsa, sizeof sa); hipMalloc(&dsb, sizeof sb);
  hipMalloc(&dc, N * sizeof(f4));
  f4 out[N];
  auto run = [&]() {
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipMemcpy(dsa, sa, sizeof sa, hipMemcpyHostToDevice);
    hipMemcpy(dsb, sb, sizeof sb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dc);
    hipMemcpy(out, dc, sizeof out, hipMemcpyDeviceToHost);
  };
  auto total = [&]() {
    double s = 0;
    for (int l = 0; l < N; ++l)
      for (int i = 0; i < 4; ++i) s += out[l][i];
    return s;
  };
  const int one = 0x38383838;  // four e4m3 1.0
  int bad = 0;
  for (int side = 0; side < 2; ++side) {
    printf("%s operand: (lane, quarter) -> lanes whose scale multiplies it\n", side ? "B" : "A");
    for (int L = 0; L < N; ++L) {
      printf("  L%2d:", L);
      for (int h = 0; h < 4; ++h) {
        for (int l = 0; l < N; ++l)
          for (int j = 0; j < 8; ++j) {
            (side ? ha : hb)[l][j] = one;  // the other operand: all 1.0
            (side ? hb : ha)[l][j] = (l == L && j / 2 == h) ? one : 0;
          }
        for (int l = 0; l < N; ++l) sa[l] = sb[l] = 0x7f7f7f7f;
        run();
        const double base = total();
        printf(" h%d[", h);
        int hits = 0;
        for (int Ls = 0; Ls < N; ++Ls) {
          for (int l = 0; l < N; ++l) sa[l] = sb[l] = 0x7f7f7f7f;
          (side ? sb : sa)[Ls] = (int)0x80808080;
          run();
          if (total() > 1.5 * base) {
            printf("%s%d", hits ? "," : "", Ls);
            if (Ls != L % 16 + 16 * (2 * (h >> 1) + ((L / 16) >> 1))) ++bad;
            ++hits;
          }
        }
        if (hits != 1) ++bad;
        printf("]");
      }
      printf("\n");
    }
  }
  // which byte does opsel 0 read: scale of lane 0 with only byte k = 128
  for (int l = 0; l < N; ++l)
    for (int j = 0; j < 8; ++j) ha[l][j] = hb[l][j] = one;
  for (int k = 0; k < 4; ++k) {
    for (int l = 0; l < N; ++l) sa[l] = sb[l] = 0x7f7f7f7f;
    run();
    const double base = total();
    sa[0] = (int)(0x7f7f7f7fu + (1u << (8 * k)));
    run();
    printf("opsel 0, A scale byte %d of lane 0 = 128: total %s\n", k, total() > base ? "changes" : "unchanged");
  }
  printf(bad ? "MAPPING DIFFERS from r + 16(2(h>>1) + (j>>1)) (%d)\n" : "quarter h of lane r+16j scaled by lane r + 16(2(h>>1) + (j>>1))\n", bad);
  return bad ? 1 : 0;
}
