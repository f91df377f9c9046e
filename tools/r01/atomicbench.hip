// atomicbench — how float-atomic row updates behave when the rows are Zipf-hot.
//
// Every wave adds a 300-float delta (one dword per lane, 5 contiguous 256-B
// instructions) to rows drawn from p(r) ~ r^-0.75 over V rows (the unigram^0.75
// negative-sampling law), the way the training kernel's hot-row path does.
// Variants: rows at their natural (contiguous) addresses, and the K hottest
// rows split into R replicas placed far apart (wave w adds to replica w % R).
// Prints row-updates/s and added GB/s per variant.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__global__ __launch_bounds__(256) void add_rows(float* M, long pitch, int d, const unsigned* rows, long per_wave,
                                                int K, int R, long rep_base, long rep_stride, int plain) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + threadIdx.x / 64;
  const unsigned* my = rows + wave * per_wave;
  const int rep = (int)(wave % R);
  for (long k = 0; k < per_wave; ++k) {
    const long r = my[k];
    float* p = (r < K && R > 1) ? M + (rep_base + (long)rep * rep_stride + r) * pitch : M + r * pitch;
    for (int v = 0; v < 5; ++v) {
      const int e = lane + 64 * v;
      if (e < d) {
        if (plain) p[e] += 1e-6f;
        else (void)__hip_atomic_fetch_add(p + e, 1e-6f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

int main(int argc, char** argv) {
  const long V = argc > 1 ? std::atol(argv[1]) : 740000;
  const int d = 300;
  const long pitch = 320;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const long blocks = ncu * 4L, waves = blocks * 4, per_wave = 512;
  // Zipf(0.75) row draws
  std::vector<double> cdf(V);
  double acc = 0;
  for (long r = 0; r < V; ++r) cdf[r] = (acc += std::pow((double)(r + 1), -0.75));
  std::vector<unsigned> h((size_t)(waves * per_wave));
  unsigned long long s = 0x9E3779B97F4A7C15ull;
  for (auto& x : h) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) / 9007199254740992.0 * acc;
    x = (unsigned)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
  }
  const int R = 16, K = 64;
  const long rep_stride = 1 << 16;  // replicas 64K rows (80 MB) apart
  const long rows_alloc = V + (long)R * rep_stride + K;
  float* M;
  unsigned* rows;
  CK(hipMalloc(&M, rows_alloc * pitch * sizeof(float)));
  CK(hipMemset(M, 0, rows_alloc * pitch * sizeof(float)));
  CK(hipMalloc(&rows, h.size() * 4));
  CK(hipMemcpy(rows, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct Var { const char* name; int K, R, plain; } vars[] = {
      {"plain_rmw", 0, 1, 1}, {"atomic_contiguous", 0, 1, 0}, {"atomic_top64_x4", K, 4, 0},
      {"atomic_top64_x16", K, 16, 0}, {"atomic_top1024_x16", 1024, 16, 0}};
  for (auto& vr : vars) {
    const long base = V;  // replicas live after the matrix
    hipLaunchKernelGGL(add_rows, dim3(blocks), dim3(256), 0, 0, M, pitch, d, rows, per_wave, vr.K, vr.R, base,
                       rep_stride / 16 * 16 > vr.K ? rep_stride : vr.K, vr.plain);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(add_rows, dim3(blocks), dim3(256), 0, 0, M, pitch, d, rows, per_wave, vr.K, vr.R, base,
                       rep_stride, vr.plain);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double n = (double)waves * per_wave;
    std::printf("{\"variant\": \"%s\", \"V\": %ld, \"ms\": %.3f, \"row_updates_per_s\": %.3e, \"added_GBps\": %.1f}\n",
                vr.name, V, ms, n / (ms * 1e-3), n * d * 4 / (ms * 1e-3) / 1e9);
  }
  return 0;
}
