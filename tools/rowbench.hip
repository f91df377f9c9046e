// rowbench — speed-of-light probe for the training kernel's memory shape.
//
// Random embedding rows of `dim` fp32 (pitch round_up(dim,32)) gathered with
// the kernel's lane layout (float4 per lane, 1-KiB wave instructions), MAXT
// rows in flight per wave, from a table far larger than the Infinity Cache:
//   gather : read rows, reduce (reads only)          -> read ceiling, FETCH_SIZE calibration
//   rmw    : read rows, add, write back (Hogwild)    -> read+write ceiling of the update
// Prints one JSON line per mode. Build: hipcc --offload-arch=gfx950 -O3 tools/rowbench.hip -o rowbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

template <int VPL, int MAXT, bool WRITE>
__global__ __launch_bounds__(256) void rows_kernel(float* M, long pitch, int d4, const unsigned* idx,
                                                   long rows_per_wave, float* sink) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const unsigned* my = idx + wave * rows_per_wave;
  float acc = 0.f;
  for (long r0 = 0; r0 < rows_per_wave; r0 += MAXT) {
    float4 v[MAXT][VPL];
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      const float* p = M + (long)my[r0 + t] * pitch;
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        const int e = 4 * (lane + 64 * k);
        v[t][k] = (e < d4) ? *reinterpret_cast<const float4*>(p + e) : make_float4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        acc += v[t][k].x + v[t][k].y + v[t][k].z + v[t][k].w;
        if (WRITE) {
          v[t][k].x += 1e-7f; v[t][k].y += 1e-7f; v[t][k].z += 1e-7f; v[t][k].w += 1e-7f;
          const int e = 4 * (lane + 64 * k);
          if (e < d4) *reinterpret_cast<float4*>(M + (long)my[r0 + t] * pitch + e) = v[t][k];
        }
      }
    }
  }
  if (acc == 12345.678f) sink[wave] = acc;
}

int main(int argc, char** argv) {
  const int dim = argc > 1 ? std::atoi(argv[1]) : 300;
  const long nrows = argc > 2 ? std::atol(argv[2]) : 3000000;  // 3.84 GB at dim 300
  const int d4 = (dim + 3) & ~3;
  const long pitch = (dim + 31) & ~31;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = ncu * 8;  // 8 x 256 threads per CU = 32 waves per CU upper bound
  const long waves = (long)blocks * 4;
  const long rows_per_wave = 6 * 400;
  float* M;
  unsigned* idx;
  float* sink;
  CK(hipMalloc(&M, nrows * pitch * sizeof(float)));
  CK(hipMemset(M, 0, nrows * pitch * sizeof(float)));
  CK(hipMalloc(&sink, waves * sizeof(float)));
  std::vector<unsigned> h((size_t)(waves * rows_per_wave));
  unsigned long long s = 88172645463325252ull;
  for (auto& x : h) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    x = (unsigned)(s % (unsigned long long)nrows);
  }
  CK(hipMalloc(&idx, h.size() * sizeof(unsigned)));
  CK(hipMemcpy(idx, h.data(), h.size() * sizeof(unsigned), hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double rows_total = (double)waves * rows_per_wave;
  for (int mode = 0; mode < 2; ++mode) {
    auto fn = mode == 0 ? &rows_kernel<2, 6, false> : &rows_kernel<2, 6, true>;
    if (d4 <= 256) fn = mode == 0 ? &rows_kernel<1, 6, false> : &rows_kernel<1, 6, true>;
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, M, pitch, d4, idx, rows_per_wave, sink);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, M, pitch, d4, idx, rows_per_wave, sink);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    const double bytes = rows_total * dim * 4.0 * (mode == 0 ? 1 : 2);
    std::printf("{\"mode\": \"%s\", \"dim\": %d, \"rows\": %.0f, \"table_GB\": %.2f, \"ms\": %.3f, "
                "\"algorithmic_GBps\": %.1f, \"rows_per_s\": %.3e}\n",
                mode == 0 ? "gather" : "rmw", dim, rows_total, nrows * pitch * 4.0 / 1e9, best,
                bytes / (best * 1e-3) / 1e9, rows_total / (best * 1e-3));
  }
  return 0;
}
