// Launch-order microbenchmark (round 5, the overlapped-steps question): how soon does a kernel start
// after the one it depends on ends, for
//   same   : B behind A on one stream (the AQL barrier bit)
//   anyord : B behind A on one stream, launched with hipExtAnyOrderLaunch (does B start before A ends?)
//   event  : A on stream 0, event, stream 1 waits for it, B on stream 1
//   free   : A on stream 0, B on stream 1, no dependency (do they run concurrently?)
// A spins ~20 us on one workgroup (a stand-in for a dW launch), B is one workgroup that records its
// start.  Times from s_memrealtime (100 MHz), medians over 200 trials.
//   hipcc --offload-arch=gfx950 -O3 -o xstream scripts/ubench/xstream.hip && ./xstream
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                      \
      return 1;                                                               \
    }                                                                         \
  } while (0)

// A: records its start and end; spins `ticks` of the 100 MHz clock on every wave
__global__ void kA(unsigned long long* t, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    t[0] = t0;
    t[1] = __builtin_amdgcn_s_memrealtime();
  }
}
// B: records its start
__global__ void kB(unsigned long long* t) {
  if (threadIdx.x == 0 && blockIdx.x == 0) t[2] = __builtin_amdgcn_s_memrealtime();
}

int main() {
  unsigned long long* d;
  CK(hipMalloc(&d, 64));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const char* names[] = {"same", "anyord", "event", "free"};
  for (int mode = 0; mode < 4; ++mode) {
    std::vector<double> gap, dur;
    for (int it = 0; it < 220; ++it) {
      hipLaunchKernelGGL(kA, dim3(64), dim3(256), 0, s0, d, 2000ull);  // 20 us
      if (mode == 0) hipLaunchKernelGGL(kB, dim3(1), dim3(64), 0, s0, d);
      if (mode == 1) hipExtLaunchKernelGGL(kB, dim3(1), dim3(64), 0, s0, nullptr, nullptr, hipExtAnyOrderLaunch, d);
      if (mode == 2) {
        CK(hipEventRecord(ev, s0));
        CK(hipStreamWaitEvent(s1, ev, 0));
        hipLaunchKernelGGL(kB, dim3(1), dim3(64), 0, s1, d);
      }
      if (mode == 3) hipLaunchKernelGGL(kB, dim3(1), dim3(64), 0, s1, d);
      CK(hipDeviceSynchronize());
      unsigned long long h[3];
      CK(hipMemcpy(h, d, 24, hipMemcpyDeviceToHost));
      if (it >= 20) {
        gap.push_back(((double)h[2] - (double)h[1]) * 0.01);  // B's start after A's end, us
        dur.push_back(((double)h[1] - (double)h[0]) * 0.01);
      }
    }
    std::sort(gap.begin(), gap.end());
    std::sort(dur.begin(), dur.end());
    std::printf("%-7s B start - A end: median %7.2f us  p10 %7.2f  p90 %7.2f   (A %.2f us)\n", names[mode],
                gap[gap.size() / 2], gap[gap.size() / 10], gap[gap.size() * 9 / 10], dur[dur.size() / 2]);
  }
  return 0;
}
