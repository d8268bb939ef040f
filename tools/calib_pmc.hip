// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the chain uses
// (MI355X_MICROARCH.md: "Other access widths are uncalibrated: calibrate on a known byte count in your own
// access pattern").  Each kernel moves exactly BYTES bytes; compare with the counters.
//   hipcc -O3 --offload-arch=gfx950 tools/calib_pmc.hip -o tools/calib_pmc
//   rocprofv3 --pmc FETCH_SIZE -- tools/calib_pmc ; rocprofv3 --pmc WRITE_SIZE -- tools/calib_pmc
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t BYTES = 1ull << 30;  // 1 GiB per kernel (beyond the 256 MiB Infinity Cache)

template <typename T>
__global__ void rd(const T* __restrict__ a, size_t n, float* __restrict__ sink) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = a[i];
    acc += reinterpret_cast<const float*>(&v)[0];
  }
  if (acc == 1234.5f) sink[0] = acc;
}

template <typename T>
__global__ void wr(T* __restrict__ a, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v;
    reinterpret_cast<float*>(&v)[0] = (float)i;
    a[i] = v;
  }
}

// emit-like: each block writes CHUNK consecutive 4-byte items starting at an arbitrary (unaligned) offset
__global__ void wr_runs(int* __restrict__ a, size_t nrun, int chunk) {
  const size_t base = (size_t)blockIdx.x * chunk + (blockIdx.x * 37) % 61;  // unaligned run starts
  if ((size_t)blockIdx.x >= nrun) return;
  for (int k = threadIdx.x; k < chunk; k += blockDim.x) a[base + k] = k;
}

int main() {
  char* buf;
  float* sink;
  if (hipMalloc(&buf, BYTES + (1 << 20)) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
  hipMemset(buf, 0, BYTES);
  const dim3 g(4096), b(256);
  hipLaunchKernelGGL(rd<float4>, g, b, 0, 0, (const float4*)buf, BYTES / 16, sink);
  hipLaunchKernelGGL(rd<float2>, g, b, 0, 0, (const float2*)buf, BYTES / 8, sink);
  hipLaunchKernelGGL(rd<float>, g, b, 0, 0, (const float*)buf, BYTES / 4, sink);
  hipLaunchKernelGGL(wr<float4>, g, b, 0, 0, (float4*)buf, BYTES / 16);
  hipLaunchKernelGGL(wr<float2>, g, b, 0, 0, (float2*)buf, BYTES / 8);
  hipLaunchKernelGGL(wr<float>, g, b, 0, 0, (float*)buf, BYTES / 4);
  const int chunk = 1536;  // ~ entries per emit block
  hipLaunchKernelGGL(wr_runs, dim3((unsigned)(BYTES / 4 / (chunk + 64))), b, 0, 0, (int*)buf, BYTES / 4 / (chunk + 64),
                     chunk);
  hipDeviceSynchronize();
  printf("each kernel moves %zu bytes (wr_runs: %zu)\n", BYTES, (BYTES / 4 / (chunk + 64)) * chunk * 4);
  return 0;
}
