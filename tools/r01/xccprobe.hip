// Probe: which XCC (HW_REG_XCC_ID) each workgroup of a grid runs on.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
  if (threadIdx.x == 0) o[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
}
int main() {
  const int n = 1024;
  int* d;
  hipMalloc(&d, n * sizeof(int));
  hipLaunchKernelGGL(k, dim3(n), dim3(128), 0, 0, d);
  int h[n];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int hist[16] = {0};
  for (int i = 0; i < n; ++i) hist[h[i] & 15]++;
  for (int x = 0; x < 16; ++x) printf("xcc %d: %d\n", x, hist[x]);
  printf("first 16 blocks:");
  for (int i = 0; i < 16; ++i) printf(" %d", h[i]);
  printf("\n");
  return 0;
}
