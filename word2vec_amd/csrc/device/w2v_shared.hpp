// w2v_shared.hpp — the shared-negatives minibatch skip-gram kernel (BASELINE
// configs[4]: SGNS with negatives shared by a window, dim 512, neg 15) on the
// gfx950 matrix cores.
//
// The update (restated sequentially in oracle/w2v_oracle.cpp:sgsn_sentence,
// which cites the reference lines it keeps): for a kept center c with window
// [lo, hi), the M <= 16 unique context ids u (multiplicity m_u) are the inputs
// (W rows) and the T <= 16 outputs t are c itself (label 1) plus the window's
// shared negative draws (label 0, C rows). Then
//   L = W_in C_out^T            (M x T, contraction over d)
//   E[u][t] = m_u (label_t - sigma(L[u][t])) alpha
//   dW_in = E C_out,  dC_out = E^T W_in      (pre-update rows)
// three small dense GEMMs — the only place in the hot path where MFMA pays.
//
// How it maps to MI355X:
//   * one workgroup of 4 wavefronts per center; wave w owns the column slice
//     [16 KB w, 16 KB (w + 1)) of every row (KB 16-column blocks). All four
//     walk the same sentence with identical (Philox) decisions.
//   * v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation): 16 rows
//     of W_in and 16 rows of C_out fit one tile, neg 15 + the center = 16.
//     Rows are gathered straight into the A/B fragment layout: lane (col =
//     lane & 15, q = lane >> 4) holds row `col`, columns 16 kb + 4q .. +3 (one
//     16-B load per block; 16 rows x 64 contiguous B per wave instruction).
//   * L: 4 MFMAs per block; the four waves' partial L tiles meet in LDS (one
//     barrier per center, double-buffered).
//   * dW^T = C^T E^T and dC^T = W^T E come out of the MFMA directly in the
//     gather layout (so the update is a register add and the write-back the
//     same 16-B stores as the gather); their A operands need the rows with
//     the column index on lane & 15, produced per block by a 16x16 transpose
//     through 2.5 KiB of per-wave LDS (row stride 20 floats: conflict-free).
//   * Hogwild across workgroups (plain read-modify-write stores), exactly as
//     the per-pair kernel's default class of rows.
#pragma once
#include "w2v_kernels.hpp"

namespace w2v {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kSnWaves = 4;     // wavefronts per workgroup (column slices)
constexpr int kSnTile = 16;     // MFMA tile edge: context rows, output rows
constexpr int kSnStride = 20;   // transpose block row stride in floats

struct SnShared {
  f32x4 part[2][kSnWaves][kWave];                // partial L tiles, by center parity
  float tr[kSnWaves][2][kSnTile * kSnStride];    // per-wave transpose blocks (W, C)
  uint32_t item[2];                              // dequeued work item, by sentence parity
  float alpha[2];
};

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Keep this wave's LDS accesses in program order (the LDS unit serves one
// wave's operations in order; this only stops the compiler reordering them).
__device__ __forceinline__ void wave_lds_order() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

// g of Word2Vec.cpp:263-264 for one (input, output) pair: f = sigma(L) through
// double as there, g = (label - f) * alpha.
__device__ __forceinline__ float sn_grad(float l, bool positive, float alpha) {
  const float e = expf(-l);
  const float f = (float)(1.0 / (double)(1.0f + e));
  return ((positive ? 1.0f : 0.0f) - f) * alpha;
}

template <int KB>
__device__ __forceinline__ void sn_center(const TrainArgs& a, SnShared& sh, int wave, int lane,
                                          const int32_t* sent, int len, int i, int c, int rw, uint32_t s,
                                          float alpha, int& par, Counters& cnt) {
  const int q = lane >> 4, col = lane & 15;
  const int lo = max(0, i - a.window + rw), hi = min(len, i + a.window + 1 - rw);
  const int span = hi - lo, me = i - lo;
  const bool valid = lane < span && lane != me;
  const int id = valid ? sent[lo + lane] : -1;
  // unique context ids (first occurrence) and their multiplicities
  bool dup = !valid;
  int mult = 0;
  for (int j = 0; j < span; ++j) {
    const int v = readlane_i(id, j);
    if (j != me && v == id) {
      mult += 1;
      dup = dup || (j < lane);
    }
  }
  const unsigned long long uniq = ballot(!dup);
  const int M = __popcll(uniq);
  if (M == 0) return;  // workgroup-uniform
  int in_l = 0, m_l = 0;
  {
    unsigned long long m = uniq;
    for (int t = 0; m; ++t) {
      const int b = __builtin_ctzll(m);
      m &= m - 1;
      const int v = readlane_i(id, b), mm = readlane_i(mult, b);
      if (lane == t) { in_l = v; m_l = mm; }
    }
  }
  // outputs: lane 0 the center, lane t in [1, K] the (t-1)-th shared draw
  const int K = a.negative;
  int neg_l = 0;
  if (lane < K) neg_l = (int)a.table[philox_table_pos(a, s, (uint32_t)i, 0u, (uint32_t)lane)];
  const int prev_draw = __shfl(neg_l, (lane + kWave - 1) & (kWave - 1));  // every lane takes part
  const int out_l = (lane == 0) ? c : prev_draw;
  bool ok = (lane == 0) || (lane <= K && out_l != c);
  for (int j = 1; j < K; ++j) {
    const int v = readlane_i(out_l, j);
    ok = ok && !(j < lane && v == out_l);
  }
  const unsigned long long okm = ballot(ok);
  cnt.centers += 1;
  cnt.contexts += (unsigned long long)M;
  cnt.targets += (unsigned long long)__popcll(okm);
  cnt.draws += (unsigned long long)K;

  // gathers into the fragment layout
  const int in_row = __shfl(in_l, col), out_row = __shfl(out_l, col);
  const bool in_ok = col < M, out_ok = (okm >> col) & 1ull;
  const int64_t cb = (int64_t)wave * (kSnTile * KB) + 4 * q;
  float* wp = a.W + (int64_t)in_row * a.pitch + cb;
  float* cp = a.C + (int64_t)out_row * a.pitch + cb;
  if (a.strict) drain_vmem();  // sequential schedule: this wave's own stores land before the re-read
  f32x4 wr[KB], cr[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    wr[kb] = in_ok ? *reinterpret_cast<const f32x4*>(wp + kSnTile * kb) : f32x4{0.f, 0.f, 0.f, 0.f};
    cr[kb] = out_ok ? *reinterpret_cast<const f32x4*>(cp + kSnTile * kb) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // L (this wave's column slice), then the workgroup sum
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    acc = mfma16x16x4(wr[kb][0], cr[kb][0], acc);
    acc = mfma16x16x4(wr[kb][1], cr[kb][1], acc);
    acc = mfma16x16x4(wr[kb][2], cr[kb][2], acc);
    acc = mfma16x16x4(wr[kb][3], cr[kb][3], acc);
  }
  sh.part[par][wave][lane] = acc;
  __syncthreads();
  // lane holds L[4q + r][col]; Lt[s] = L[col][4q + s] (same sums, same order)
  f32x4 L = sh.part[par][0][lane];
#pragma unroll
  for (int w = 1; w < kSnWaves; ++w) L += sh.part[par][w][lane];
  float Lt[4];
  {
    const float* pf = reinterpret_cast<const float*>(&sh.part[par][0][0]);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int idx = (((col >> 2) * 16 + 4 * q + s4) << 2) + (col & 3);
      float v = pf[idx];
#pragma unroll
      for (int w = 1; w < kSnWaves; ++w) v += pf[w * kWave * 4 + idx];
      Lt[s4] = v;
    }
  }
  par ^= 1;
  // E in both layouts: Ea[r] = E[4q + r][col], Et[s] = E[col][4q + s]
  float Ea[4], Et[4];
  const int m_col = __shfl(m_l, col);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int u = 4 * q + r;
    const int m_u = __shfl(m_l, u);
    const bool pair_a = u < M && ((okm >> col) & 1ull);
    Ea[r] = pair_a ? (float)m_u * sn_grad(L[r], col == 0, alpha) : 0.f;
    const int t = 4 * q + r;
    const bool pair_t = col < M && ((okm >> t) & 1ull);
    Et[r] = pair_t ? (float)m_col * sn_grad(Lt[r], t == 0, alpha) : 0.f;
  }
  // dW^T = C^T E^T and dC^T = W^T E per 16-column block, added in place
  float* tw = sh.tr[wave][0];
  float* tc = sh.tr[wave][1];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    *reinterpret_cast<f32x4*>(tw + col * kSnStride + 4 * q) = wr[kb];
    *reinterpret_cast<f32x4*>(tc + col * kSnStride + 4 * q) = cr[kb];
    wave_lds_order();
    float wd[4], cd[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      wd[s4] = tw[(4 * q + s4) * kSnStride + col];  // W[4q + s][16 kb + col]
      cd[s4] = tc[(4 * q + s4) * kSnStride + col];  // C[4q + s][16 kb + col]
    }
    wave_lds_order();
    f32x4 dw = {0.f, 0.f, 0.f, 0.f}, dc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      dw = mfma16x16x4(cd[s4], Et[s4], dw);  // dW[col][16 kb + 4q + r]
      dc = mfma16x16x4(wd[s4], Ea[s4], dc);  // dC[col][16 kb + 4q + r]
    }
    wr[kb] += dw;
    cr[kb] += dc;
    if (in_ok) *reinterpret_cast<f32x4*>(wp + kSnTile * kb) = wr[kb];
    if (out_ok) *reinterpret_cast<f32x4*>(cp + kSnTile * kb) = cr[kb];
  }
}

// Epoch kernel: workgroups dequeue sentences (Word2Vec.cpp:375-394) and walk
// them with the reference's subsampling and window shrink (Philox draws).
template <int KB>
__global__ __launch_bounds__(kSnWaves * kWave) void train_shared_neg_kernel(TrainArgs a) {
  __shared__ SnShared sh;
  const int lane = lane_id();
  const int wave = (int)(threadIdx.x >> 6);
  Counters cnt;
  int par = 0;
  float alpha0 = a.init_alpha;  // thread 0's schedule state
  bool first = true;
  const uint32_t wmax = (uint32_t)(a.window < 1 ? 1 : a.window);
  for (int it = 0;; ++it) {
    const int slot = it & 1;
    if (threadIdx.x == 0) {
      const uint32_t k = atomicAdd(a.work, 1u);
      sh.item[slot] = k;
      if ((int64_t)k < a.n_sent) {
        if (a.fixed_alpha > 0.0f) {
          alpha0 = a.fixed_alpha;
        } else if (first || (k % 10u) == 0u) {
          const unsigned long long cw = __hip_atomic_load(a.words, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const float al = (float)(a.init_alpha * (1.0 - 1.0 / a.iter * (double)cw / a.train_words));
          alpha0 = (a.min_alpha < al) ? al : a.min_alpha;
          first = false;
        }
      }
      sh.alpha[slot] = alpha0;
    }
    __syncthreads();
    const uint32_t k = sh.item[slot];
    if ((int64_t)k >= a.n_sent) break;
    const float alpha = sh.alpha[slot];
    const int64_t s = a.order ? a.order[k] : (int64_t)k;
    if (s < 0 || s >= a.n_corpus) continue;
    const int64_t base = a.soff[s];
    const int len = (int)(a.soff[s + 1] - base);
    const int32_t* sent = a.ids + base;
    for (int i0 = 0; i0 < len; i0 += kWave) {
      const int ii = i0 + lane;
      const bool in = ii < len;
      const int c_l = in ? sent[ii] : 0;
      const float p_l = in ? a.keep[c_l] : 0.f;
      uint32_t o0, o1, o2, o3;
      philox((uint32_t)ii, (uint32_t)s, 0xFFFFFFFFu, a.epoch, a.key0, a.key1, o0, o1, o2, o3);
      const float u_l = canonical_f(o0);
      const int rw_l = (int)(((uint64_t)o1 * wmax) >> 32);
      unsigned long long kept = ballot(in && !(p_l < u_l));
      while (kept) {
        const int b = __builtin_ctzll(kept);
        kept &= kept - 1;
        sn_center<KB>(a, sh, wave, lane, sent, len, i0 + b, readlane_i(c_l, b), readlane_i(rw_l, b), (uint32_t)s,
                      alpha, par, cnt);
      }
    }
    if (threadIdx.x == 0) atomicAdd(a.words, (unsigned long long)len);
    cnt.sentences += 1;
  }
  if (threadIdx.x == 0) {  // every wave counted the same centers; wave 0 reports
    atomicAdd(&a.stats[0], cnt.centers);
    atomicAdd(&a.stats[1], cnt.contexts);
    atomicAdd(&a.stats[2], cnt.targets);
    atomicAdd(&a.stats[3], cnt.draws);
    atomicAdd(&a.stats[4], cnt.sentences);
  }
}

}  // namespace w2v
