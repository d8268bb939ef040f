// Placement probe: which XCD / CU each block of a 512 x 512-thread grid (72 KiB LDS, as k_rds_class) lands on.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ __launch_bounds__(512) void probe(int* out, int spin) {
  extern __shared__ float lds[];
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  lds[threadIdx.x] = (float)threadIdx.x;
  long long t0 = clock64();
  while (clock64() - t0 < spin) {}
  __syncthreads();
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x] = (int)(xcc & 0xf);
    out[3 * blockIdx.x + 1] = (int)((hw >> 8) & 0xf) | (((hw >> 13) & 0x7) << 4);  // CU id | SE id << 4
    out[3 * blockIdx.x + 2] = (int)lds[5];
  }
}
int main() {
  const int nb = 512;
  int* d;
  hipMalloc(&d, nb * 3 * sizeof(int));
  hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 72 * 1024, 0, d, 200000);
  std::vector<int> h(nb * 3);
  hipMemcpy(h.data(), d, nb * 3 * sizeof(int), hipMemcpyDeviceToHost);
  int mism = 0;
  for (int b = 0; b < nb; ++b) mism += (h[3 * b] != h[(b % 8) * 3]);
  printf("blocks whose XCD != XCD of block (b %% 8): %d of %d\n", mism, nb);
  for (int b = 0; b < 80; ++b) printf("b%d:x%d/c%02x ", b, h[3 * b], h[3 * b + 1]);
  printf("\n");
  // CU sharing: for each (xcc, cu-id) pair list blocks
  for (int b = 0; b < 16; ++b) {
    printf("block %d shares its CU with:", b);
    for (int c = 0; c < nb; ++c)
      if (c != b && h[3 * c] == h[3 * b] && h[3 * c + 1] == h[3 * b + 1]) printf(" %d", c);
    printf("\n");
  }
  return 0;
}
