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
//   * one workgroup of NW wavefronts per center; wave w owns the column slice
//     [16 KB w, 16 KB (w + 1)) of every row (KB 16-column blocks, NW * KB * 16
//     = the row pitch). All NW walk the same sentence with identical (Philox)
//     decisions. Two waves per center keep the per-center bookkeeping
//     (window dedup, draws) from being repeated on every SIMD while letting
//     four workgroups (four centers' gathers) share a CU.
//   * v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulation): 16 rows
//     of W_in and 16 rows of C_out fit one tile, neg 15 + the center = 16.
//     Rows are gathered straight into the A/B fragment layout: lane (col =
//     lane & 15, q = lane >> 4) holds row `col`, columns 16 kb + 4q .. +3 (one
//     16-B load per block; 16 rows x 64 contiguous B per wave instruction).
//     Unused slots point at slot 0's row (same addresses as lane col 0: no
//     extra traffic), so no load sits behind a branch; E masks them out.
//   * L: 4 MFMAs per block; the waves' partial L tiles meet in LDS (one
//     barrier per center, double-buffered). E = f(L) is evaluated once per
//     element and transposed through LDS.
//   * dW^T = C^T E^T and dC^T = W^T E come out of the MFMA directly in the
//     gather layout (so the update is a register add and the write-back the
//     same 16-B stores as the gather); their A operands need the rows with
//     the column index on lane & 15, produced per block by a 16x16 transpose
//     through per-wave LDS (row stride 20 floats: conflict-free reads).
//   * windows are word2vec.c's (and pWord2Vec's): subsampled tokens leave the
//     sentence, so a window spans kept tokens. Each wave compacts the kept
//     tokens into an LDS ring (ballot + mbcnt) and stages the unigram-table
//     draws (dependent random HBM reads) of a batch of up to 64 centers with
//     one wait; a center then issues no memory operation before its gathers.
//   * Hogwild across workgroups (read-modify-write), the frequent rows with
//     device-coherent (sc1) loads and write-through stores: see rows_rsrc.
#pragma once
#include "w2v_kernels.hpp"

namespace w2v {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kSnTile = 16;     // MFMA tile edge: context rows, output rows
constexpr int kSnStride = 20;   // transpose block row stride in floats
constexpr int kSnRing = 256;    // kept-token ring (holds a 64-center batch, its lookahead and one more block)

// Private output rows: each workgroup accumulates its updates of the P most
// frequent C rows (the negatives every center draws) in LDS and writes them
// back every a.flush_every centers, instead of a coherent read-modify-write
// of those few rows by every center (their write-through traffic serialises
// on a handful of memory channels: measured, 16 coherent rows cost a third of
// the throughput). The row slots fill kSnPrivBytes of LDS, at most 32 rows.
template <int KB, int NW>
constexpr int kSnPriv = (kSnPrivBytes / (NW * KB * 64)) < 32 ? (kSnPrivBytes / (NW * KB * 64)) : 32;

template <int KB, int NW>
struct SnShared {
  f32x4 part[2][NW][kWave];                      // partial L tiles, by center parity
  f32x4 e[NW][kWave];                            // per-wave E tile (for its transpose)
  float tr[NW][2][kSnTile * kSnStride];          // per-wave transpose block [W, C] (one buffer: see the update loop)
  // written identically by every wave (read only before the per-center
  // barrier, rewritten only after it): the kept tokens of the sentence (ring,
  // by kept index) and the draws of a batch of <= 64 centers
  int ring_id[kSnRing];
  int ring_pos[kSnRing];                         //   positions in the sentence
  int ring_rw[kSnRing];                          //   window shrinks
  int draw[kWave][kSnTile];                      // [center in batch][k]
  float priv[kSnPriv<KB, NW>][NW * KB * kSnTile];  // pending deltas of C rows [0, P); wave w owns its columns
  uint32_t item[2];                              // dequeued work item, by sentence parity
  float alpha[2];
};

// Phase timing (diagnostic builds only: make prof, -DW2V_SN_PROF=1; tools/sn_prof.sh).
struct SnProf {
#ifdef W2V_SN_PROF
  unsigned long long t = 0, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  __device__ void stamp(int k) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    acc[k] += now - t;
    t = now;
  }
#else
  __device__ void stamp(int) {}
#endif
};

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Row traffic of the frequent rows is device-coherent. Per-XCD L2s are not
// coherent with each other inside a launch (MI355X_MICROARCH.md, XCD): with
// plain (write-back) stores every XCD keeps training its own L2-resident
// version of the rows it touches constantly, and the versions are merged line
// by line at write-back (measured: analogy accuracy collapses to ~0 as soon
// as workgroups span two XCDs). Rows below a.hot_wc (the vocab is sorted by
// count: the rows an L2 could keep resident) are loaded with sc1 (skips the
// CU's L1, which other CUs' stores never refresh) and stored with sc1
// (write-through: the line leaves the writer's L2), so a copy lives in an L2
// only between one read and that workgroup's write-back. Rarer rows are
// evicted from any L2 long before their next use and keep the cached path.
// Measured alternatives: per-XCD replicas merged between
// launches diverge (summed deltas) or under-train (averaged).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, -1, 0x00020000);
}
constexpr int kSc1 = 16;  // buffer cache-policy bit: sc1 (device scope)
__device__ __forceinline__ f32x4 load_row4(__amdgpu_buffer_rsrc_t r, uint32_t off, bool coherent) {
  if (coherent) return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1);
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ void store_row4(f32x4 v, __amdgpu_buffer_rsrc_t r, uint32_t off, bool coherent) {
  if (coherent && !(W2V_EXP_SKIP & 32)) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kSc1);
  else __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}

template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false); }

// Write back two consecutive 16-column blocks (lo = block 2j, hi = block 2j+1,
// fragment layout: lane (col, q) holds row col, columns 4q..4q+3 of each) as
// two instructions of 8 rows x 128 contiguous bytes, so that a write-through
// (sc1) store sends whole lines to memory instead of 64-B halves. Lane col and its partner col ^ 8 (DPP row_ror:8)
// trade their hi blocks: instruction 0 writes rows 0..7, instruction 1 rows 8..15.
__device__ __forceinline__ void store_pair(f32x4 lo, f32x4 hi, __amdgpu_buffer_rsrc_t r, uint32_t off, bool ok, bool coh,
                                           int col) {
  f32x4 hp;
#pragma unroll
  for (int e = 0; e < 4; ++e) hp[e] = __int_as_float(dpp_i<0x128>(__float_as_int(hi[e])));
  const uint32_t off_p = (uint32_t)dpp_i<0x128>((int)off) + 64u;  // partner row, block 2j+1
  const bool ok_p = dpp_i<0x128>((int)ok) != 0, coh_p = dpp_i<0x128>((int)coh) != 0;
  const bool low = col < 8;
  // instruction 0: rows 0..7 — own lo for col < 8, the partner's hi for col >= 8
  if (low ? ok : ok_p) store_row4(low ? lo : hp, r, low ? off : off_p, low ? coh : coh_p);
  // instruction 1: rows 8..15 — own lo for col >= 8, the partner's hi for col < 8
  if (low ? ok_p : ok) store_row4(low ? hp : lo, r, low ? off_p : off, low ? coh_p : coh);
}

// Gather two consecutive 16-column blocks (block 2j, 2j+1) as two
// instructions of 8 rows x 128 contiguous bytes (store_pair's inverse):
// instruction 0 reads rows 0..7 — lane col < 8 its own block 2j, lane col >= 8
// the block 2j+1 of row col - 8 (its partner col ^ 8) — instruction 1 rows
// 8..15 the same way. The raw results land in (t0, t1); pair_fixup later puts
// the lane's own blocks there (own block 2j from whichever instruction read
// it, own block 2j+1 from the partner through DPP row_ror:8), after the loads
// have been issued for every block.
__device__ __forceinline__ void load_pair(f32x4& t0, f32x4& t1, __amdgpu_buffer_rsrc_t r, uint32_t off, bool coh,
                                          int col) {
  const uint32_t off_p = (uint32_t)dpp_i<0x128>((int)off) + 64u;  // partner row, block 2j+1
  const bool coh_p = dpp_i<0x128>((int)coh) != 0;
  const bool low = col < 8;
  t0 = load_row4(r, low ? off : off_p, low ? coh : coh_p);
  t1 = load_row4(r, low ? off_p : off, low ? coh_p : coh);
}
__device__ __forceinline__ void pair_fixup(f32x4& t0, f32x4& t1, int col) {
  const bool low = col < 8;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float own = low ? t0[e] : t1[e];
    const float other = low ? t1[e] : t0[e];  // the partner's block 2j+1
    t0[e] = own;
    t1[e] = __int_as_float(dpp_i<0x128>(__float_as_int(other)));
  }
}

// Keep this wave's LDS accesses in program order (the LDS unit serves one
// wave's operations in order; this only stops the compiler reordering them).
__device__ __forceinline__ void wave_lds_order() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

// g of Word2Vec.cpp:263-264 for one (input, output) pair: f = sigma(L) with
// the reference's rounding (ns_sigmoid), g = (label - f) * alpha.
__device__ __forceinline__ float sn_grad(float l, bool positive, float alpha) {
  const float e = expf(-l);
  const float f = ns_sigmoid(e);
  return ((positive ? 1.0f : 0.0f) - f) * alpha;
}

// Center t (kept index) of the sentence's kept tokens; its window spans kept
// indices [t - window + rw, t + window + 1 - rw) clipped to [0, nk) (word2vec.c
// windows: subsampled tokens are gone from the sentence, as in pWord2Vec).
// Slot b (< 64) of the staged draws belongs to it.
template <int KB, int NW>
__device__ __forceinline__ void sn_center(const TrainArgs& a, SnShared<KB, NW>& sh, __amdgpu_buffer_rsrc_t rW,
                                          __amdgpu_buffer_rsrc_t rC, int wave, int lane, int t, int nk, int b,
                                          float alpha, int& par, Counters& cnt, SnProf& pf_, unsigned& dirty) {
  pf_.stamp(0);
  const int q = lane >> 4, col = lane & 15;
  const int c = sh.ring_id[t & (kSnRing - 1)], rw = sh.ring_rw[t & (kSnRing - 1)];
  const int lo = max(0, t - a.window + rw), hi = min(nk, t + a.window + 1 - rw);
  const int span = hi - lo;
  const int wv = sh.ring_id[(lo + lane) & (kSnRing - 1)];
  const int id = (lane < span && lo + lane != t) ? wv : -1;
  // unique context ids (first occurrence) and their multiplicities
  bool dup = id < 0;
  int mult = 0;
  for (int j = 0; j < span; ++j) {
    const int v = readlane_i(id, j);
    if (v == id) {
      mult += 1;
      dup = dup || (j < lane);
    }
  }
  const unsigned long long uniq = ballot(!dup);
  const int M = __popcll(uniq);
  if (M == 0) return;  // workgroup-uniform (a one-token sentence)
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
  // W row gathers (slot col, or slot 0's row for an unused slot)
  const bool in_ok = col < M;
  const int in_row = __shfl(in_l, in_ok ? col : 0);
  const int64_t cb = (int64_t)wave * (kSnTile * KB) + 4 * q;
  const uint32_t wo = (uint32_t)(((int64_t)in_row * a.pitch + cb) * 4);  // byte offsets (< 4 GiB, host-checked)
  const bool w_coh = in_row < a.hot_wc;
  const bool w_atom = in_row < a.hot_atomic;
  if (a.strict) drain_vmem();  // sequential schedule: this wave's own stores land before the re-read
  f32x4 wr[KB], cr[KB];
#pragma unroll
  for (int kb = 0; kb < KB; kb += 2) load_pair(wr[kb], wr[kb + 1], rW, wo + 64u * kb, w_coh, col);
  // outputs: lane 0 the center, lane t in [1, K] the (t-1)-th shared draw
  const int K = a.negative;
  const int prev_draw = sh.draw[b][(lane + kSnTile - 1) & (kSnTile - 1)];
  const int out_l = (lane == 0) ? c : prev_draw;
  bool ok = (lane == 0) || (lane <= K && out_l != c);
  for (int j = 1; j < K; ++j) {
    const int v = readlane_i(out_l, j);
    ok = ok && !(j < lane && v == out_l);
  }
  const unsigned long long okm = ballot(ok);
  const bool out_ok = (okm >> col) & 1ull;
  const int out_row = __shfl(out_l, out_ok ? col : 0);
  const uint32_t co = (uint32_t)(((int64_t)out_row * a.pitch + cb) * 4);
  const bool c_coh = out_row < a.hot_wc;
  const bool c_priv = out_row < a.priv_n;  // this workgroup's pending delta lives in LDS
  const bool c_atom = !c_priv && out_row < a.hot_atomic;
  float* pr = &sh.priv[c_priv ? out_row : 0][(int)cb];
  if (a.priv_n > 0) {  // this wave's dirty private rows (lanes 0..15 hold the 16 output slots)
    unsigned long long pm = ballot(c_priv && out_ok && lane < kSnTile);
    while (pm) {
      const int bb = __builtin_ctzll(pm);
      pm &= pm - 1;
      dirty |= 1u << readlane_i(out_row, bb);
    }
  }
#pragma unroll
  for (int kb = 0; kb < KB; kb += 2) load_pair(cr[kb], cr[kb + 1], rC, co + 64u * kb, c_coh, col);
  cnt.centers += 1;
  cnt.contexts += (unsigned long long)M;
  cnt.targets += (unsigned long long)__popcll(okm);
  cnt.draws += (unsigned long long)K;
  pf_.stamp(1);
#pragma unroll
  for (int kb = 0; kb < KB; kb += 2) {
    pair_fixup(wr[kb], wr[kb + 1], col);
    pair_fixup(cr[kb], cr[kb + 1], col);
  }
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  if (c_priv) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) cr[kb] += *reinterpret_cast<const f32x4*>(pr + kSnTile * kb);
  }
  // unused slots hold slot 0's row: finite, and every E term that touches them
  // is masked to zero below, so they add nothing to dW, dC (and are not stored)
  pf_.stamp(2);
  // L (this wave's column slice), then the workgroup sum
  f32x4 acc = zero;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    acc = mfma16x16x4(wr[kb][0], cr[kb][0], acc);
    acc = mfma16x16x4(wr[kb][1], cr[kb][1], acc);
    acc = mfma16x16x4(wr[kb][2], cr[kb][2], acc);
    acc = mfma16x16x4(wr[kb][3], cr[kb][3], acc);
  }
  sh.part[par][wave][lane] = acc;
  pf_.stamp(3);
  __syncthreads();
  pf_.stamp(4);
  // lane holds L[4q + r][col] (the partials summed in wave order: the same
  // value in every wave); E once per element, Et[s] = E[col][4q + s] by LDS
  f32x4 L = sh.part[par][0][lane];
#pragma unroll
  for (int w = 1; w < NW; ++w) L += sh.part[par][w][lane];
  par ^= 1;
  if (wave == 0 && out_ok && 4 * q < M) {  // divergence: a non-finite sigma argument (kNonFinite)
    bool bad = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) bad = bad || (4 * q + r < M && !__builtin_isfinite(L[r]));
    if (bad) atomicAdd(a.stats + kNonFinite, 1ull);
  }
  f32x4 Ea;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int u = 4 * q + r;
    const int m_u = __shfl(m_l, u);
    Ea[r] = (u < M && out_ok) ? (float)m_u * sn_grad(L[r], col == 0, alpha) : 0.f;
  }
  sh.e[wave][lane] = Ea;
  wave_lds_order();
  // contraction step s of dW covers outputs 4s + q, of dC inputs 4s + q, so the
  // steps past the last output (K + 1) or the last input (M) are skipped
  float Eo[4], Ei[4];
  {
    const float* pe = reinterpret_cast<const float*>(&sh.e[wave][0]);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      Eo[s4] = pe[((((col >> 2) << 4) + 4 * s4 + q) << 2) + (col & 3)];  // E[col][4s + q]
      Ei[s4] = pe[((col + 16 * s4) << 2) + q];                            // E[4s + q][col]
    }
  }
  const int n_out = (K + 1 + 3) >> 2, n_in = (M + 3) >> 2;
  // Atomic rows (below a.hot_atomic): their deltas are staged in the free
  // private-row slots of LDS (this wave's columns) and added to HBM row-wise
  // after the update, 256 contiguous bytes per atomic instruction; rows past
  // the free slots fall back to the coherent store.
  const int n_slots = kSnPriv<KB, NW> - a.priv_n;
  const unsigned long long atw = ballot(w_atom && in_ok && lane < kSnTile);
  const unsigned long long atc = ballot(c_atom && out_ok && lane < kSnTile);
  const unsigned long long below = (1ull << col) - 1ull;
  int w_slot = (w_atom && in_ok) ? __popcll(atw & below) : n_slots;
  int c_slot = (c_atom && out_ok) ? __popcll(atw) + __popcll(atc & below) : n_slots;
  const bool w_stage = w_slot < n_slots, c_stage = c_slot < n_slots;
  float* ws = &sh.priv[a.priv_n + (w_stage ? w_slot : 0)][(int)cb];
  float* cs = &sh.priv[a.priv_n + (c_stage ? c_slot : 0)][(int)cb];
  pf_.stamp(5);
  // dW^T = C^T E^T and dC^T = W^T E per 16-column block, added in place.
  // Block kb + 1 is written into the same transpose buffer right after block
  // kb's reads are issued: one wave's LDS operations execute in order, so the
  // reads return block kb (the fence only keeps the compiler from reordering;
  // no wait). One buffer instead of two frees 5 KiB per workgroup for two
  // more LDS row slots (kSnPrivBytes).
  float* const tw0 = sh.tr[wave][0];
  float* const tc0 = sh.tr[wave][1];
  *reinterpret_cast<f32x4*>(tw0 + col * kSnStride + 4 * q) = wr[0];
  *reinterpret_cast<f32x4*>(tc0 + col * kSnStride + 4 * q) = cr[0];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    wave_lds_order();
    float wd[4], cd[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      wd[s4] = tw0[(4 * s4 + q) * kSnStride + col];  // W[4s + q][16 kb + col]
      cd[s4] = tc0[(4 * s4 + q) * kSnStride + col];  // C[4s + q][16 kb + col]
    }
    wave_lds_order();
    if (kb + 1 < KB) {
      *reinterpret_cast<f32x4*>(tw0 + col * kSnStride + 4 * q) = wr[kb + 1];
      *reinterpret_cast<f32x4*>(tc0 + col * kSnStride + 4 * q) = cr[kb + 1];
    }
    f32x4 dw = zero, dc = zero;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      if (s4 < n_out) dw = mfma16x16x4(cd[s4], Eo[s4], dw);  // dW[col][16 kb + 4q + r]
      if (s4 < n_in) dc = mfma16x16x4(wd[s4], Ei[s4], dc);   // dC[col][16 kb + 4q + r]
    }
    wr[kb] += dw;
    cr[kb] += dc;
    if (c_priv && out_ok) *reinterpret_cast<f32x4*>(pr + kSnTile * kb) += dc;
    if (w_stage) *reinterpret_cast<f32x4*>(ws + kSnTile * kb) = dw;
    if (c_stage) *reinterpret_cast<f32x4*>(cs + kSnTile * kb) = dc;
    if (kb & 1) {  // blocks kb - 1, kb written back as whole 128-B lines
      store_pair(wr[kb - 1], wr[kb], rW, wo + 64u * (kb - 1), in_ok && !w_stage, w_coh, col);
      store_pair(cr[kb - 1], cr[kb], rC, co + 64u * (kb - 1), out_ok && !c_priv && !c_stage, c_coh, col);
    }
  }
  {  // the staged atomic rows, row by row
    constexpr int kCols = KB * kSnTile;
    wave_lds_order();
    unsigned long long mw = atw, mc = atc;
    for (int sl = 0; sl < n_slots && (mw | mc); ++sl) {
      const bool is_w = mw != 0;
      const int bb = __builtin_ctzll(is_w ? mw : mc);
      if (is_w) mw &= mw - 1; else mc &= mc - 1;
      const int64_t row = readlane_i(is_w ? in_row : out_row, bb);
      float* dst = (is_w ? a.W : a.C) + row * a.pitch + wave * kCols;
      const float* src = &sh.priv[a.priv_n + sl][wave * kCols];
#pragma unroll
      for (int cc = 0; cc < kCols; cc += kWave)
        if (cc + lane < kCols)
          if (!(W2V_EXP_SKIP & 8))
            (void)__hip_atomic_fetch_add(dst + cc + lane, src[cc + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    wave_lds_order();
  }
  pf_.stamp(7);
  pf_.stamp(6);
}

// Move this wave's columns of its dirty private rows' pending deltas into C
// with memory-side float atomics (no update lost between workgroups) and clear
// them, each row scaled by a.priv_sc (the per-pair kernel's flush_private
// averaging, w2v_kernels.hpp: a fixed function of the row's frequency rank,
// computed on the host per launch).
template <int KB, int NW>
__device__ __forceinline__ void sn_flush_private(const TrainArgs& a, SnShared<KB, NW>& sh, int wave, int lane,
                                                 unsigned& dirty) {
  constexpr int kCols = KB * kSnTile;  // this wave's columns of a row
  unsigned m = (unsigned)__builtin_amdgcn_readfirstlane((int)dirty);
  dirty = 0;
  if (m == 0) return;
  wave_lds_order();
  while (m) {
    const int r = __builtin_ctz(m);
    m &= m - 1;
    const float sc = a.priv_sc[r];
    float* dst = a.C + (int64_t)r * a.pitch + wave * kCols;
    for (int cc = lane; cc < kCols; cc += kWave) {
      float* p = &sh.priv[r][wave * kCols + cc];
      const float v = *p;
      *p = 0.f;
      if (v != 0.f && !(W2V_EXP_SKIP & 16))
        (void)__hip_atomic_fetch_add(dst + cc, v * sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  wave_lds_order();
}

// Epoch kernel: workgroups dequeue sentences (Word2Vec.cpp:375-394) and walk
// them with the reference's subsampling and window shrink (Philox draws).
template <int KB, int NW, int WAVES_PER_SIMD>
__global__ __launch_bounds__(NW * kWave, WAVES_PER_SIMD) void train_shared_neg_kernel(TrainArgs a) {
  __shared__ SnShared<KB, NW> sh;
  const int lane = lane_id();
  const int wave = (int)(threadIdx.x >> 6);
  Counters cnt;
  SnProf prof;
#ifdef W2V_SN_PROF
  prof.t = __builtin_amdgcn_s_memtime();
#endif
  const __amdgpu_buffer_rsrc_t rW = rows_rsrc(a.W), rC = rows_rsrc(a.C);
  int par = 0;
  int since_flush = 0;  // centers since the private rows were written back
  unsigned dirty = 0;  // private rows: this wave's dirty mask
  if (a.priv_n > 0) {
    for (int k = threadIdx.x; k < kSnPriv<KB, NW> * NW * KB * kSnTile; k += blockDim.x) (&sh.priv[0][0])[k] = 0.f;
    __syncthreads();
  }
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
        } else if (first || ((a.item0 + k) % 10) == 0) {
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
    const int64_t s = a.order ? a.order[a.item0 + k] : a.item0 + (int64_t)k;
    if (s < 0 || s >= a.n_corpus) continue;
    const int64_t base = a.soff[s];
    const int len = (int)(a.soff[s + 1] - base);
    const int32_t* sent = a.ids + base;
    // Produce kept tokens into the ring 64 positions at a time; consume them
    // in batches of <= 64 centers once each batch's windows (window kept
    // tokens past its last center) are in the ring, or the sentence is done.
    int nk = 0, t_done = 0, i0 = 0;
    for (;;) {
      while (i0 < len && nk < t_done + kWave + a.window) {
        const int ii = i0 + lane;
        const bool in = ii < len;
        const int c_l = in ? sent[ii] : 0;
        const float p_l = in ? a.keep[c_l] : 0.f;
        uint32_t o0, o1, o2, o3;
        philox((uint32_t)ii, (uint32_t)s, 0xFFFFFFFFu, a.epoch, a.key0, a.key1, o0, o1, o2, o3);
        const float u_l = canonical_f(o0);
        const int rw_l = (int)(((uint64_t)o1 * wmax) >> 32);
        const bool keep_l = in && !(p_l < u_l);
        const unsigned long long kept = ballot(keep_l);
        if (keep_l) {
          const int r = (nk + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(kept >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((unsigned)kept, 0u))) &
                        (kSnRing - 1);
          sh.ring_id[r] = c_l;
          sh.ring_pos[r] = ii;
          sh.ring_rw[r] = rw_l;
        }
        nk += __popcll(kept);
        i0 += kWave;
      }
      const int n_batch = min(kWave, (i0 >= len ? nk : nk - a.window) - t_done);
      if (n_batch <= 0) {
        if (i0 >= len) break;
        continue;
      }
      wave_lds_order();
      {  // stage the batch's table draws: lane l -> center t_done + l
        int dv[kSnTile];
        const int pos = sh.ring_pos[(t_done + lane) & (kSnRing - 1)];
#pragma unroll
        for (int kk = 0; kk < kSnTile; ++kk) {
          dv[kk] = 0;
          if (lane < n_batch && kk < a.negative)
            dv[kk] = (int)a.table[philox_table_pos(a, (uint32_t)s, (uint32_t)pos, 0u, (uint32_t)kk)];
        }
#pragma unroll
        for (int kk = 0; kk < kSnTile; kk += 4)
          *reinterpret_cast<int4*>(&sh.draw[lane][kk]) = make_int4(dv[kk], dv[kk + 1], dv[kk + 2], dv[kk + 3]);
        wave_lds_order();
      }
      for (int b = 0; b < n_batch; ++b) {
        sn_center<KB, NW>(a, sh, rW, rC, wave, lane, t_done + b, nk, b, alpha, par, cnt, prof, dirty);
        if (a.priv_n > 0 && ++since_flush >= a.flush_every) {
          sn_flush_private<KB, NW>(a, sh, wave, lane, dirty);
          since_flush = 0;
        }
      }
      t_done += n_batch;
    }
    if (threadIdx.x == 0) atomicAdd(a.words, (unsigned long long)len);
    cnt.sentences += 1;
  }
  if (a.priv_n > 0) sn_flush_private<KB, NW>(a, sh, wave, lane, dirty);
#ifdef W2V_SN_PROF
  prof.stamp(0);
  if (lane == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2))
    printf("SNPROF block %u wave %d centers %llu sent %llu: %llu %llu %llu %llu %llu %llu %llu %llu\n", blockIdx.x,
           wave, cnt.centers, cnt.sentences, prof.acc[0], prof.acc[1], prof.acc[2], prof.acc[3], prof.acc[4],
           prof.acc[5], prof.acc[6], prof.acc[7]);
#endif
  if (threadIdx.x == 0) {  // every wave counted the same centers; wave 0 reports
    atomicAdd(&a.stats[0], cnt.centers);
    atomicAdd(&a.stats[1], cnt.contexts);
    atomicAdd(&a.stats[2], cnt.targets);
    atomicAdd(&a.stats[3], cnt.draws);
    atomicAdd(&a.stats[4], cnt.sentences);
  }
}

}  // namespace w2v

