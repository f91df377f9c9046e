// Float atomic adds on a few hot rows, every workgroup adding: device-scope
// (memory-side) into one copy vs workgroup-scope into a per-XCD copy (indexed
// by HW_REG_XCC_ID). Checks that no add is lost in either form and times them.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/atomic_scope_bench tools/atomic_scope_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kRowFloats = 256;

__device__ __forceinline__ int xcc_id() {
  return (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7);  // HW_REG_XCC_ID, 4 bits
}

template <int SCOPE>
__global__ void add_rows(float* dst, int rows, int iters, int per_xcd) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float* base = dst + (per_xcd ? (size_t)xcc_id() * rows * kRowFloats : 0);
  for (int it = 0; it < iters; ++it) {
    const int row = (it * 7 + blockIdx.x * 3 + wave) % rows;
    float* p = base + (size_t)row * kRowFloats + lane;
#pragma unroll
    for (int v = 0; v < 4; ++v) (void)__hip_atomic_fetch_add(p + 64 * v, 1.0f, __ATOMIC_RELAXED, SCOPE);
  }
}

__global__ void which_xcc(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

int main() {
  const int rows = 64, iters = 2000, blocks = 1024, threads = 256;
  float* d = nullptr;
  int* x = nullptr;
  hipMalloc(&d, 8 * rows * kRowFloats * sizeof(float));
  hipMalloc(&x, blocks * sizeof(int));
  hipLaunchKernelGGL(which_xcc, dim3(blocks), dim3(64), 0, 0, x);
  std::vector<int> xs(blocks);
  hipMemcpy(xs.data(), x, blocks * sizeof(int), hipMemcpyDeviceToHost);
  int hist[8] = {0};
  for (int v : xs) hist[v & 7]++;
  printf("blocks per xcc id:");
  for (int k = 0; k < 8; ++k) printf(" %d", hist[k]);
  printf("\n");
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double expect = (double)blocks * (threads / 64) * iters * 4 * 64;  // adds of 1.0
  for (int mode = 0; mode < 3; ++mode) {
    hipMemset(d, 0, 8 * rows * kRowFloats * sizeof(float));
    hipEventRecord(e0);
    if (mode == 0) hipLaunchKernelGGL(add_rows<__HIP_MEMORY_SCOPE_AGENT>, dim3(blocks), dim3(threads), 0, 0, d, rows, iters, 0);
    if (mode == 1) hipLaunchKernelGGL(add_rows<__HIP_MEMORY_SCOPE_WORKGROUP>, dim3(blocks), dim3(threads), 0, 0, d, rows, iters, 1);
    if (mode == 2) hipLaunchKernelGGL(add_rows<__HIP_MEMORY_SCOPE_AGENT>, dim3(blocks), dim3(threads), 0, 0, d, rows, iters, 1);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<float> h(8 * rows * kRowFloats);
    hipMemcpy(h.data(), d, h.size() * sizeof(float), hipMemcpyDeviceToHost);
    double sum = 0;
    for (float f : h) sum += f;
    const char* name[] = {"agent scope, one copy", "workgroup scope, per-XCD copies", "agent scope, per-XCD copies"};
    printf("%-34s %8.3f ms  %.2f G adds/s  sum %.0f of %.0f (%s)\n", name[mode], ms, expect / (ms * 1e6), sum, expect,
           sum == expect ? "exact" : "LOST");
  }
  return 0;
}
