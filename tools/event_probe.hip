// event_probe.hip — what a hipEvent pair around a kernel measures on this ROCm (VERDICT r4 "next" #3).
// Build: hipcc -O2 --offload-arch=gfx950 tools/event_probe.hip -o tools/event_probe
// Run on the GPU box, alone and under `rocprofv3 --kernel-trace --stats`, and compare:
//   case 1  one stream:   e0 | X (spin 2 ms) | e1 | Y (spin 0.2 ms) | e2
//   case 2  two streams:  A: X (spin 3 ms), evA        B: wait(evA) | e0 | Y (spin 0.2 ms) | e1
//           (the question: does e0 take its time stamp when B passes the wait, or earlier?)
//   case 3  as case 2 with device time stamps: B: wait(evA) | stamp | Y | stamp (a one-lane kernel writing
//           wall_clock64() with a vector store), the time between the stamps, and the hipExtLaunchKernelGGL
//           start / stop events of Y.
// Every kernel is short and bounded (spin on the 100 MHz wall clock with a fixed deadline).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void spin(long long ticks, int* out) {  // ticks of the 100 MHz wall clock
  const long long t0 = wall_clock64();
  long long t = t0;
  while (t - t0 < ticks) t = wall_clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = (int)(t - t0);
}

__global__ void stamp(long long* buf, int i) {
  if (threadIdx.x == 0) buf[i] = wall_clock64();
}

static float ms(hipEvent_t a, hipEvent_t b) {
  float m = 0.f;
  CK(hipEventElapsedTime(&m, a, b));
  return m;
}

int main() {
  int* out;
  long long* ts;
  CK(hipMalloc(&out, 4096 * sizeof(int)));
  CK(hipMalloc(&ts, 64 * sizeof(long long)));
  hipStream_t A, B;
  CK(hipStreamCreate(&A));
  CK(hipStreamCreate(&B));
  hipEvent_t e[8];
  for (auto& x : e) CK(hipEventCreate(&x));
  const dim3 g(1024), b(64);  // 1024 one-wave blocks: every CU busy, room left for other kernels
  for (int rep = 0; rep < 3; ++rep) {
    // case 1
    CK(hipEventRecord(e[0], A));
    hipLaunchKernelGGL(spin, g, b, 0, A, 200000LL, out);  // 2 ms
    CK(hipEventRecord(e[1], A));
    hipLaunchKernelGGL(spin, g, b, 0, A, 20000LL, out);  // 0.2 ms
    CK(hipEventRecord(e[2], A));
    CK(hipDeviceSynchronize());
    printf("case1 rep %d: e0-e1 (X 2 ms) %.3f  e1-e2 (Y 0.2 ms) %.3f ms\n", rep, ms(e[0], e[1]), ms(e[1], e[2]));
    // case 2
    hipLaunchKernelGGL(spin, g, b, 0, B, 1000LL, out);  // something earlier on B (10 us)
    CK(hipStreamSynchronize(B));
    hipLaunchKernelGGL(spin, g, b, 0, A, 300000LL, out);  // 3 ms
    CK(hipEventRecord(e[3], A));
    CK(hipStreamWaitEvent(B, e[3], 0));
    CK(hipEventRecord(e[4], B));
    hipLaunchKernelGGL(spin, g, b, 0, B, 20000LL, out);  // 0.2 ms
    CK(hipEventRecord(e[5], B));
    CK(hipDeviceSynchronize());
    printf("case2 rep %d: B wait|e0|Y 0.2 ms|e1: e0-e1 %.3f ms (A's 3 ms kernel ended %.3f ms after e0)\n", rep,
           ms(e[4], e[5]), ms(e[4], e[3]));
    // case 3
    hipLaunchKernelGGL(spin, g, b, 0, B, 1000LL, out);
    CK(hipStreamSynchronize(B));
    hipLaunchKernelGGL(spin, g, b, 0, A, 300000LL, out);
    CK(hipEventRecord(e[3], A));
    CK(hipStreamWaitEvent(B, e[3], 0));
    hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, B, ts, 0);
    hipExtLaunchKernelGGL(spin, g, b, 0, B, e[6], e[7], 0, 20000LL, out);
    hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, B, ts, 1);
    CK(hipDeviceSynchronize());
    long long h[2];
    CK(hipMemcpy(h, ts, sizeof h, hipMemcpyDeviceToHost));
    printf("case3 rep %d: stamps around Y %.3f ms, hipExtLaunchKernelGGL events of Y %.3f ms\n", rep,
           (h[1] - h[0]) * 1e-5, ms(e[6], e[7]));
  }
  printf("done\n");
  return 0;
}
