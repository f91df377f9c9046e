// LDS accumulate microbenchmark (gfx950): the cost of adding a wave's 64
// floats (one lane each, contiguous) into an LDS row, the operation the
// per-pair kernels use for their privatised rows' pending deltas (priv_add:
// ds_add_f32), against the alternatives. 16-wave workgroups, one per CU,
// every wave adds `iters` times into row (wave % rows) of `rows` LDS rows.
//   mode 0  ds_add_f32 (atomicAdd on __shared__ float)
//   mode 1  ds_add_u32 (atomicAdd on __shared__ unsigned)
//   mode 2  ds_read_b32 + v_add + ds_write_b32 (non-atomic read-modify-write)
//   mode 3  ds_add_rtn_f32 (the returning form)
//   mode 4  ds_write_b32 only (store bound)
// build: hipcc --offload-arch=gfx950 -O3 -o lds_atomic_bench tools/lds_atomic_bench.hip
// usage: ./lds_atomic_bench   (prints cycles per wave-instruction per CU)
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(1024) void bench(int iters, int rows, float* out, unsigned long long* cyc) {
  __shared__ float buf[16 * 64 * 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = threadIdx.x; k < 16 * 64 * 4; k += blockDim.x) buf[k] = 0.f;
  __syncthreads();
  float* row = buf + (wave % rows) * 64 * 4 + lane;
  const float d = 1e-3f * (float)(lane + 1);
  float acc = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    float* p = row + 64 * (i & 3);
    if (MODE == 0) {
      atomicAdd(p, d);
    } else if (MODE == 1) {
      atomicAdd(reinterpret_cast<unsigned*>(p), (unsigned)(lane + 1));
    } else if (MODE == 2) {
      *(volatile float*)p = *(volatile float*)p + d;
    } else if (MODE == 3) {
      acc += atomicAdd(p, d);
    } else {
      *(volatile float*)p = d;
    }
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  if (acc == 12345.f) out[0] = acc;
  if (threadIdx.x < 64) out[blockIdx.x * 64 + threadIdx.x] = buf[threadIdx.x];
}

template <int MODE>
double run(int iters, int rows, int blocks, float* out, unsigned long long* cyc) {
  hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(1024), 0, 0, iters, rows, out, cyc);
  hipDeviceSynchronize();
  unsigned long long h[1024];
  hipMemcpy(h, cyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double s = 0;
  for (int b = 0; b < blocks; ++b) s += (double)h[b];
  // s_memtime counts at 100 MHz on gfx9 boxes? report raw units per wave-instruction of the CU
  return s / blocks / ((double)iters * 16.0);
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 1024 * 64 * sizeof(float));
  hipMalloc(&cyc, 1024 * sizeof(unsigned long long));
  const int blocks = 256, iters = 4096;
  const char* names[] = {"ds_add_f32", "ds_add_u32", "read+write", "ds_add_rtn_f32", "write only"};
  for (int rows : {1, 16}) {
    double r[5];
    r[0] = run<0>(iters, rows, blocks, out, cyc);
    r[1] = run<1>(iters, rows, blocks, out, cyc);
    r[2] = run<2>(iters, rows, blocks, out, cyc);
    r[3] = run<3>(iters, rows, blocks, out, cyc);
    r[4] = run<4>(iters, rows, blocks, out, cyc);
    for (int m = 0; m < 5; ++m)
      printf("{\"rows\": %d, \"mode\": \"%s\", \"memtime_per_wave_instr_per_cu\": %.3f}\n", rows, names[m], r[m]);
  }
  return 0;
}
