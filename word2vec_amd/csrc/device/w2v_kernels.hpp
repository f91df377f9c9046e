// w2v_kernels.hpp — gfx950 (CDNA4) training kernels for the Word2Vec hot path.
//
// What they compute is the reference's per-sentence update, unchanged:
//   skip-gram  Word2Vec.cpp:319-353 (center W row is the input, fixed over the
//              window; each context word is predicted; W[center] += grad once)
//   CBOW       Word2Vec.cpp:273-317 (sum of C rows over the SET of context ids,
//              /n if cbow_mean; scatter grad back to every unique id)
//   NS         Word2Vec.cpp:251-271 (unique negatives from the unigram table,
//              the positive overrides a colliding negative)
//   HS         Word2Vec.cpp:232-249 (walk the Huffman path of the predicted word)
// and the epoch loop Word2Vec.cpp:371-395 (sentences in the shuffled order,
// alpha recomputed from the shared word counter every 10th sentence).
//
// How they map to MI355X:
//   * one 64-lane wavefront owns one sentence at a time and walks it in order,
//     exactly like one OpenMP thread of the reference; wavefronts dequeue
//     sentences from a global head counter (Hogwild across sentences, as the
//     reference is across threads). A one-wave grid is the deterministic
//     sequential schedule used for parity.
//   * an embedding row is spread over the wave one dword per lane per 64
//     elements (element lane + 64 v): every row gather is NV fully coalesced
//     256-B wave instructions, and a row update is NV 256-B contiguous
//     instructions — the shape at which MI355X float atomics run at full rate.
//     The rows of all targets of one context (<= MAXT) are gathered together.
//   * dot products reduce across the wave with DPP (row rotations + row
//     broadcasts, no LDS), the result read back with v_readlane into an SGPR,
//     so the sigmoid and gradient scalar are wave-uniform.
//   * updates `row += g * x` (and W[center] += grad, C[ctx] += grad) are
//     either plain stores of the updated row (lock-free Hogwild) or memory-side
//     global_atomic_add_f32 of g * x — the same fp32 rounding as the
//     reference's `row = row + g*x`, but no update is lost when thousands of
//     wavefronts hit one row. Rows inside the "hot" range (frequent words: the
//     low vocab indices, the top of the Huffman tree) take the atomic path;
//     their gathers use L1-bypassing agent-scope loads so a wavefront sees its
//     own atomics. Per-XCD L2s are not coherent inside a launch, so what
//     another XCD wrote may be read late (delayed SGD) but is never lost.
//   * Philox4x32-10 counter-based draws make every random decision a pure
//     function of (key, epoch, sentence, position, slot, k); in Philox mode
//     subsampling decisions for 64 tokens are made at once (one lane per
//     token) and only kept centers are walked. Replay mode consumes the
//     reference's own mt19937 stream recorded on the host, in its draw order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace w2v {

constexpr int kWave = 64;
// Timing-only experiment builds (tools/r02/exp_variant.sh; never the product):
// bit 1 skips the hot-row atomics of the targets, bit 2 the global atomics of
// the private-row flushes, bit 4 the hot context-row atomics of CBOW; in the
// shared-negatives kernel bit 8 skips the staged atomic rows, bit 16 the
// private-row flush atomics, bit 32 makes the coherent (sc1) stores plain;
// bit 64 skips the per-pair kernels' plain (Hogwild) row stores, bit 128
// the LDS adds into the private rows' pending deltas, bit 256 the private
// rows' pending-delta reads.
#ifndef W2V_EXP_SKIP
#define W2V_EXP_SKIP 0
#endif
// Largest workgroup per row width: up to 16 waves share one LDS region of
// privatised rows while the register budget (<=128 VGPRs at 4 waves/SIMD)
// holds; wider rows keep 4-wave workgroups.
template <int NV>
constexpr int kMaxBlock = NV <= 6 ? 1024 : 256;
// Waves per SIMD the epoch kernel is compiled for: two 16-wave workgroups per
// CU when a row is <= 2 floats per lane (d <= 128: 64 VGPRs), else one.
#ifndef W2V_MIN_WAVES
template <int NV>
constexpr int kMinWaves = NV <= 2 ? 8 : NV <= 16 ? 4 : 2;  // d > 1024: 256 VGPRs
#else  // occupancy experiments (tools/r02/occ_probe.sh)
template <int NV>
constexpr int kMinWaves = W2V_MIN_WAVES;
#endif

struct TrainArgs {
  float* W;
  float* C;
  float* S;             // synapses1
  int64_t pitch;        // row pitch in floats (multiple of 4)
  int32_t dim;          // word_dim
  int32_t window;
  int32_t negative;
  int32_t cbow_mean;
  int32_t iter;
  float init_alpha;
  float min_alpha;
  double train_words;
  const int32_t* ids;
  const int64_t* soff;
  const int64_t* order;  // sentence ids to visit; null = identity over all sentences
  int64_t n_sent;        // entries of `order` to process (work items)
  int64_t n_corpus;      // sentences in the corpus (ids from `order` outside it are skipped)
  const float* keep;
  const uint32_t* table;
  int64_t table_size;
  const uint8_t* codes;
  const int32_t* points;
  const int64_t* coff;
  const uint32_t* replay;      // replay stream
  const int64_t* replay_off;   // per sentence, this epoch
  unsigned long long* words;   // progress (current_words)
  unsigned int* work;          // dequeue head
  unsigned long long* stats;   // centers, contexts, targets, draws, sentences
  uint32_t key0, key1, epoch;
  float fixed_alpha;           // > 0: use instead of the schedule
  // Row bounds are 32-bit (ids are int32): a row index read back from a lane
  // sits in an SGPR, and gfx950's scalar unit compares 32-bit values only
  // (64-bit bounds moved every hot / private test onto the VALU).
  int32_t hot_wc;              // W / C rows [0, hot_wc) update with atomics (shared-negatives: sc1 traffic)
  int32_t hot_s;               // synapses1 rows [hot_s, V-1) update with atomics
  const float* hot_sc;         // per hot node j >= hot_s: its deltas' scale, hot_sc[j - hot_s] (null: 1; hot_node_scales)
  int32_t strict;              // 1: drain own atomics before re-reading (sequential schedule)
  const float* priv_M;         // output matrix whose hottest rows are privatised in LDS (or null)
  int32_t priv_lo;             // privatised rows [priv_lo, priv_lo + priv_n)
  int32_t priv_n;
  float priv_avg;              // > 0: average, not sum, the workgroups' deltas of a privatised row (see flush_private)
  int32_t flush_every;         // the privatised deltas are flushed every this many centers of the workgroup
  const float* ctx_M;          // CBOW: context matrix whose rows [0, ctx_n) are privatised too (or null)
  int32_t ctx_n;
  int32_t ctx_flush_every;     // centers of the workgroup between flushes of the context rows
  int32_t* wide_ids;           // CBOW, window > kMaxWideWindow: per wave a slice of wide_stride ints (cbow_center_huge)
  int64_t wide_stride;
  int64_t item0;               // shared-negatives kernel: work items are order[item0 + k] (or item0 + k)
  int64_t hot_atomic;          // shared-negatives kernel: W / C rows [0, hot_atomic) take memory-side atomic deltas
  int32_t nseg;                // work items per sentence (parallel Philox schedule; 1 = whole sentences)
  int32_t seg_len;             // tokens per item when nseg > 1 (a multiple of 64)
  // Flush scales of the privatised rows (flush_private), computed on the host
  // per launch from the corpus statistics (launch_train, priv_scales): row p of
  // the output range gets priv_sc[p], row p of the context range ctx_sc[p].
  float priv_sc[128];          // kPrivMax
  float ctx_sc[64];            // kCtxMax
};

// LDS the shared-negatives kernel gives its row slots (w2v_shared.hpp kSnPriv; <= 32 rows):
// 20 KiB = 10 rows at d = 512 with four 2-wave workgroups per CU (38.9 KiB each).
#ifndef W2V_SN_PRIV_BYTES
constexpr int kSnPrivBytes = 20 * 1024;
#else  // experiments (tools/r02/sn_slots_probe.sh)
constexpr int kSnPrivBytes = W2V_SN_PRIV_BYTES;
#endif

struct Counters {
  unsigned long long centers = 0, contexts = 0, targets = 0, draws = 0, sentences = 0;
  // Phase timing (diagnostic builds only: make prof, -DW2V_PP_PROF=1;
  // tools/pp_prof.sh): s_memtime since the previous stamp, summed per phase.
#ifdef W2V_PP_PROF
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

// stats[kNonFinite] counts sigma arguments (row . input dot products) that
// were not finite: the model diverged (w2v_dev_train_epoch returns
// W2V_ERR_DIVERGED). Wave-uniform check, one atomic per offending update.
constexpr int kNonFinite = 5;
__device__ __forceinline__ void note_nonfinite(unsigned long long* stats, bool bad, int lane) {
  if (bad && lane == 0) atomicAdd(stats + kNonFinite, 1ull);
}

// ---------------------------------------------------------------------------
// Wave primitives
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

// Full-wave sum, broadcast to every lane (all 64 lanes must be active).
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xb1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4e>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x128>(v);  // row_ror:8
  v += dpp_f<0x142>(v);  // row_bcast:15
  v += dpp_f<0x143>(v);  // row_bcast:31
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }

// Wait until this wave's outstanding memory operations (incl. no-return atomics) completed.
__device__ __forceinline__ void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. SC'11), the throughput-mode RNG.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t k0, uint32_t k1, uint32_t& o0, uint32_t& o1,
                                       uint32_t& o2, uint32_t& o3) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  o0 = c0; o1 = c1; o2 = c2; o3 = c3;
}

// libstdc++ generate_canonical<float,24> of one 32-bit draw.
__device__ __forceinline__ float canonical_f(uint32_t x) {
  float r = (float)x * (1.0f / 4294967296.0f);
  return r >= 1.0f ? __int_as_float(0x3F7FFFFF) : r;
}

// Draw k of context slot `slot`: counter (position, sentence, slot << 8 | k's
// low byte, epoch ^ (k's high bits << 20)); for k < 256 (every negative up to
// 255) the last word is the epoch alone.
__device__ __forceinline__ uint32_t philox_table_pos(const TrainArgs& a, uint32_t s, uint32_t i,
                                                     uint32_t slot, uint32_t k) {
  uint32_t o0, o1, o2, o3;
  philox(i, s, (slot << 8) | (k & 255u), a.epoch ^ ((k >> 8) << 20), a.key0, a.key1, o0, o1, o2, o3);
  const uint64_t x = ((uint64_t)o1 << 32) | o0;
  return (uint32_t)__umul64hi(x, (uint64_t)a.table_size);
}

// ---------------------------------------------------------------------------
// LDS-privatised rows of the per-pair kernel (when priv_n + ctx_n > 0), per workgroup:
//   words [0,4) dirty mask of the output rows (2 x 64 bits), [4,8) of the
//   context rows, [8] centers of the workgroup, [9, 13) lock bits of the
//   output rows, [13, 15) of the context rows (W2V_PRIV_ADD 2), then (from
//   lds_header_words) the pending deltas: priv_n output rows, then ctx_n
//   context rows, NV * 64 floats each. The output range holds at most
//   kPrivMax rows, the context range kCtxMax.
// ---------------------------------------------------------------------------
constexpr int kPrivMax = 128;
constexpr int kCtxMax = 64;
__host__ __device__ inline int64_t lds_header_words(int64_t, int64_t) { return 16; }

struct PrivRows {  // one privatised row range [lo, lo + n) of matrix M (n == 0: none)
  float* delta = nullptr;
  unsigned long long* dirty = nullptr;
  unsigned* lock = nullptr;  // one bit per row (priv_lock)
  float* M = nullptr;
  int lo = 0;
  int n = 0;
  bool ctx = false;  // the context range (flush scales a.ctx_sc) or the output range (a.priv_sc)
  __device__ bool has(int row) const { return (unsigned)(row - lo) < (unsigned)n; }  // one scalar compare
};

template <int NV>
__device__ __forceinline__ PrivRows out_rows(const TrainArgs& a, float* lds) {
  PrivRows p;
  if (lds == nullptr || a.priv_n == 0) return p;
  p.dirty = reinterpret_cast<unsigned long long*>(lds);
  p.lock = reinterpret_cast<unsigned*>(lds) + 9;
  p.delta = lds + lds_header_words(a.priv_n, a.ctx_n);
  p.M = const_cast<float*>(a.priv_M);
  p.lo = a.priv_lo;
  p.n = a.priv_n;
  return p;
}

template <int NV>
__device__ __forceinline__ PrivRows ctx_rows(const TrainArgs& a, float* lds) {
  PrivRows p;
  if (lds == nullptr || a.ctx_n == 0) return p;
  p.dirty = reinterpret_cast<unsigned long long*>(lds + 4);
  p.lock = reinterpret_cast<unsigned*>(lds) + 13;
  p.delta = lds + lds_header_words(a.priv_n, a.ctx_n) + (int64_t)a.priv_n * (NV * kWave);
  p.M = const_cast<float*>(a.ctx_M);
  p.lo = 0;
  p.n = a.ctx_n;
  p.ctx = true;
  return p;
}

// ---------------------------------------------------------------------------
// Row I/O: a row is NV floats per lane, element lane + 64 v (v < NV). Rows
// are NV * 64 floats apart at least (pitch >= NV * 64, w2v_dev_bind_model)
// and their columns past word_dim are zero, and stay zero: every delta there
// is g * 0. So every lane loads, stores and adds its whole row, with no
// per-element guard: no exec-mask branches around the memory instructions
// (an exec-masked zero-fill of a register whose load may be outstanding made
// the compiler wait for ALL this wave's memory operations — vmcnt(0), stores
// and memory-side atomics included — before every hot row's gather), and
// every store writes whole 128-B lines. The dot products add the padding's
// zeros, so the sums are bit-identical to the guarded form.
// ---------------------------------------------------------------------------
#ifndef W2V_ROW_GUARDS  // timing experiments only (tools/r03): 1 = the per-element guards of round 2
#define W2V_ROW_GUARDS 0
#endif
// W2V_ROW_BOUNDED: the row's last vector (the only one holding padding) goes
// through a buffer resource whose range is the row's d floats: a lane past it
// loads 0 and stores nothing WITHOUT an exec mask and without moving the
// padding's bytes (d 100: 112 of a row's 512 B). Same values as the unbounded
// form (the padding is zero). Measured (profiles/r03t_bounded_ab.log; parity
// green): 0.2-0.3 % slower on configs[0]-[2] — the padding shares its 128-B
// line with the row's last valid floats, so no line is saved. Off.
#ifndef W2V_ROW_BOUNDED
#define W2V_ROW_BOUNDED 0
#endif
constexpr int kBufSc1 = 16;  // buffer cache-policy bit sc1: device scope (bypasses the CU's L1)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const float* base, int d) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, d * 4, 0x00020000);
}

template <int NV>
__device__ __forceinline__ void load_row(const float* M, int64_t row, int64_t pitch, int d, int lane, bool fresh,
                                         float (&r)[NV]) {
  const float* p = M + row * pitch + lane;
  constexpr int NU = W2V_ROW_BOUNDED ? NV - 1 : NV;  // vectors loaded unbounded
  if (fresh) {  // agent-scope relaxed loads: global_load_dword sc1, bypass the CU's L1
#pragma unroll
    for (int v = 0; v < NU; ++v)
      r[v] = (!W2V_ROW_GUARDS || lane + kWave * v < d)
                 ? __hip_atomic_load(p + kWave * v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                 : 0.f;
  } else {
#pragma unroll
    for (int v = 0; v < NU; ++v) r[v] = (!W2V_ROW_GUARDS || lane + kWave * v < d) ? p[kWave * v] : 0.f;
  }
  if (W2V_ROW_BOUNDED) {
    const uint32_t off = (uint32_t)(lane + kWave * (NV - 1)) * 4u;
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(M + row * pitch, d);
    r[NV - 1] = __uint_as_float(fresh ? __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, kBufSc1)
                                      : __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
  }
}

template <int NV>
__device__ __forceinline__ void store_row(float* M, int64_t row, int64_t pitch, int d, int lane,
                                          const float (&r)[NV]) {
  float* p = M + row * pitch + lane;
  constexpr int NU = W2V_ROW_BOUNDED ? NV - 1 : NV;
#pragma unroll
  for (int v = 0; v < NU; ++v)
    if (!W2V_ROW_GUARDS || lane + kWave * v < d) p[kWave * v] = r[v];
  if (W2V_ROW_BOUNDED)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r[NV - 1]), row_rsrc(M + row * pitch, d),
                                          (uint32_t)(lane + kWave * (NV - 1)) * 4u, 0, 0);
}

// row += delta, memory-side (no-return global_atomic_add_f32, 256 contiguous B
// per instruction). The padding lanes are masked here: an atomic has no
// destination register (nothing to zero-fill, no wait), and a memory-side add
// of 0 would still cost the atomic unit a request (d 300: 320 adds per row
// instead of 300; measured 2.5 % of configs[2], profiles/r03d_guards_ab.log).
// Vectors of a row every lane of which is inside word_dim: pick_nv
// (w2v_dev.hip) takes the smallest row width >= ceil(d / 64) of {1, 2, 3, 4,
// 5, 6, 8, 12, 16, 24, 32}, so d > 64 x the next smaller width and those
// vectors need no lane mask (a mask is an exec-mask round trip per atomic).
template <int NV>
constexpr int kFullVecs = NV <= 6 ? NV - 1 : NV == 8 ? 6 : NV == 12 ? 8 : NV == 16 ? 12 : NV == 24 ? 16 : 24;

template <int NV>
__device__ __forceinline__ void atomic_add_row(float* M, int64_t row, int64_t pitch, int d, int lane,
                                               const float (&delta)[NV]) {
  float* p = M + row * pitch + lane;
#pragma unroll
  for (int v = 0; v < NV; ++v)
    if (v < kFullVecs<NV> || lane + kWave * v < d)
      (void)__hip_atomic_fetch_add(p + kWave * v, delta[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// M[row] += delta: atomically for hot rows; else read-modify-write (Hogwild).
template <int NV>
__device__ __forceinline__ void add_to_row(float* M, int64_t row, bool hot, int64_t pitch, int d, int lane,
                                           const float (&delta)[NV]) {
  if (hot) {
    atomic_add_row<NV>(M, row, pitch, d, lane, delta);
  } else {
    float cur[NV];
    load_row<NV>(M, row, pitch, d, lane, false, cur);
#pragma unroll
    for (int v = 0; v < NV; ++v) cur[v] += delta[v];
    if (!(W2V_EXP_SKIP & 64)) store_row<NV>(M, row, pitch, d, lane, cur);
  }
}

// A privatised row's value is the global row plus this workgroup's pending delta.
template <int NV>
__device__ __forceinline__ void priv_read(const PrivRows& pr, int64_t row, int lane, float (&r)[NV]) {
  if (W2V_EXP_SKIP & 256) return;
  const float* q = pr.delta + (row - pr.lo) * (NV * kWave) + lane;
#pragma unroll
  for (int v = 0; v < NV; ++v) r[v] += q[kWave * v];
}

// Add delta into the row's pending delta, then mark the row dirty (after the
// adds: a wave's LDS operations are ordered).
//   W2V_PRIV_ADD 0 (rounds 1-4): ds_add_f32 per element. gfx950 runs an LDS float atomic
//     one lane at a time: 192 cycles per wave instruction against 4 for
//     ds_add_u32 and 10.5 for a ds_read + ds_write pair
//     (tools/lds_atomic_bench.hip, profiles/r05d_lds_atomic_bench.log);
//     on configs[1] these adds held ~44 % of the kernel's time (a build
//     without them: 262 -> 468 M words/s, profiles/r05c_*).
//   1: ds_read + v_add + ds_write, unguarded (timing experiments: two waves
//     of a workgroup can lose an add, and a flush racing an add counts the
//     row's delta twice).
//   2 (the default): the same read-modify-write under a per-row LDS lock bit
//     that lane 0 takes with one single-lane ds_or_rtn_b32 (a wave's own LDS
//     operations execute in order, so the release after the writes publishes
//     them); flush_private takes the same lock: exact, as the float atomics
//     are. Same box, alternating (profiles/r05e_*): configs[1] 262 -> 330-337
//     M words/s (unguarded 334-337), configs[0] / [2] unchanged, every
//     headline-scale and full-concurrency quality gate passing.
#ifndef W2V_PRIV_ADD  // 2 since round 5: configs[1] 262 -> 330-337 M words/s (profiles/r05e_2_ab_c2_lock.log)
#define W2V_PRIV_ADD 2
#endif
__device__ __forceinline__ void priv_lock(const PrivRows& pr, int p, int lane) {
  unsigned* w = pr.lock + (p >> 5);
  const unsigned bit = 1u << (p & 31);
  for (;;) {
    unsigned old = 0;
    if (lane == 0) old = atomicOr(w, bit);
    old = (unsigned)__builtin_amdgcn_readfirstlane((int)old);
    if (!(old & bit)) break;
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");  // the row's LDS reads stay after the acquire
}
__device__ __forceinline__ void priv_unlock(const PrivRows& pr, int p, int lane) {
  asm volatile("" ::: "memory");  // the row's LDS writes stay before the release
  if (lane == 0) atomicAnd(pr.lock + (p >> 5), ~(1u << (p & 31)));
}
template <int NV>
__device__ __forceinline__ void priv_add(const PrivRows& pr, int64_t row, int d, int lane, const float (&delta)[NV]) {
  const int64_t p = row - pr.lo;
  float* q = pr.delta + p * (NV * kWave) + lane;
  if (W2V_PRIV_ADD == 2) {
    priv_lock(pr, (int)p, lane);
    float cur[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) cur[v] = q[kWave * v];
#pragma unroll
    for (int v = 0; v < NV; ++v) q[kWave * v] = cur[v] + delta[v];  // padding: 0 + 0
    priv_unlock(pr, (int)p, lane);
  } else if (W2V_PRIV_ADD == 1) {
    float cur[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) cur[v] = q[kWave * v];
#pragma unroll
    for (int v = 0; v < NV; ++v) q[kWave * v] = cur[v] + delta[v];  // padding: 0 + 0
  } else {
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (!(W2V_EXP_SKIP & 128) && (v < kFullVecs<NV> || lane + kWave * v < d)) atomicAdd(q + kWave * v, delta[v]);
  }
  if (lane == 0) atomicOr(pr.dirty + (p >> 6), 1ull << (p & 63));
}

// NS's sigma, Word2Vec.cpp:263: f = 1.0 / (1 + exp(-f)) — a float sum 1 + e
// divided in double and rounded back to the float f. For a float x, the
// double quotient 1.0 / x rounded to float IS the correctly rounded float
// quotient 1.0f / x (double rounding is innocuous for division when the wider
// format has >= 2p + 2 bits, 53 >= 50; checked exhaustively for x in [1,
// 2^30)), and HIP's f32 division is correctly rounded (no fast math): the same
// bits as the f64 division at a fraction of its VALU cost.
#ifndef W2V_NS_SIGMOID_F64  // timing experiments only: 1 = the f64 division (same bits, more VALU)
__device__ __forceinline__ float ns_sigmoid(float e) { return 1.0f / (1.0f + e); }
#else
__device__ __forceinline__ float ns_sigmoid(float e) { return (float)(1.0 / (double)(1.0f + e)); }
#endif

// g of up to N targets at once (Word2Vec.cpp:240-242 HS, :263-264 NS): the
// targets' dot products f[t] are wave-uniform, so target t's sigma and g are
// evaluated in lane t — one exp / division sequence for the batch instead of
// one per target (the same operations on the same values: bit-identical);
// code_l holds target t's code (HS: the Huffman code; NS: 1 - label) in lane
// c0 + t. Returns g in lane t (read back with readlane_f).
template <bool HSF>
__device__ __forceinline__ float grad_of(float fl, int cl, float alpha) {
  const float e = expf(-fl);
#ifdef W2V_HS_F32  // timing experiments only: HS's sigma and g in f32 (not the reference's double)
  if (HSF) return (1.0f - (float)cl - 1.0f / (1.0f + e)) * alpha;
#endif
  if (HSF) {
    const float s = (float)(1.0 / (1.0 + (double)e));
    return (float)((1.0 - (double)cl - (double)s) * (double)alpha);
  }
  return ((float)(1 - cl) - ns_sigmoid(e)) * alpha;
}

template <int N, bool HSF>
__device__ __forceinline__ float batch_grad(const float (&f)[N], int T, int code_l, int c0, float alpha, int lane) {
  float fl = 0.f;
  int cl = 0;
#pragma unroll
  for (int t = 0; t < N; ++t) {
    if (t < T) {
      const int c = readlane_i(code_l, c0 + t);
      fl = (lane == t) ? f[t] : fl;
      cl = (lane == t) ? c : cl;
    }
  }
  return grad_of<HSF>(fl, cl, alpha);
}

// ---------------------------------------------------------------------------
// The dot products of a batch of targets, reduced together (W2V_BATCH_DOTS).
// One wave_sum per target costs 6 DPP adds + a readlane each, and the batch's
// sigma step then gathers the sums back into lanes (2 selects + a readlane per
// target): ~13 VALU per target on a kernel that at d = 100 keeps the VALU busy
// ~77 % of its cycles (profiles/r04c_c1_pmc_counters.json: SQ_ACTIVE_INST_VALU
// / SQ_WAVE_CYCLES per SIMD). Instead the NB (4 or 8) per-lane partials are
// folded pairwise, halving the vector count at each step:
//   xor 32  v_permlane32_swap(a, b): a = [a.lo | b.lo], b = [a.hi | b.hi];
//           a + b holds a's half-sums in lanes 0-31 and b's in lanes 32-63
//   xor 16  v_permlane16_swap (odd rows of the first operand with even rows
//           of the second): rows of a + b = [a, b, a', b'] sums
//   xor 8   keep / give selected by lane bit 3 plus a row_ror:8 DPP add
//   xor 4, 2, 1 (one vector left): quad_perm and row_half_mirror DPP adds
// so each group of 8 lanes (NB = 4: of 16) ends with one target's total:
// 18 VALU for 8 targets instead of ~104. The lanes of a group hold identical
// bits (a + b == b + a). Only the order of the 64-term sum changes.
// ---------------------------------------------------------------------------
#ifndef W2V_BATCH_DOTS
#define W2V_BATCH_DOTS 1
#endif
__device__ __forceinline__ void swap32(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
// 16-lane row r of a permlane16-folded vector holds pair member
// ((r & 1) << 1) | (r >> 1) (rows 0..3: members 0, 2, 1, 3; an involution).
__host__ __device__ constexpr int row_member(int r) { return ((r & 1) << 1) | (r >> 1); }
template <int N>
constexpr int kBatchN = N <= 4 ? 4 : 8;
// The first lane of target t's group after batch_dots<N>.
template <int N>
__device__ __forceinline__ constexpr int batch_lane(int t) {
  return kBatchN<N> == 8 ? 16 * row_member(t & 3) + 8 * (t >> 2) : 16 * row_member(t);
}
// The target whose total lane `lane` holds after batch_dots<N>.
template <int N>
__device__ __forceinline__ int batch_target(int lane) {
  return kBatchN<N> == 8 ? 4 * ((lane >> 3) & 1) + row_member(lane >> 4) : row_member(lane >> 4);
}

template <int N>
__device__ __forceinline__ float batch_dots(const float (&p)[N], int lane) {
  static_assert(N >= 1 && N <= 8, "batch of 1..8 targets");
  constexpr int NB = kBatchN<N>;
  float q[NB / 2];
#pragma unroll
  for (int k = 0; k < NB / 2; ++k) {  // xor 32
    float a = 2 * k < N ? p[2 * k] : 0.f, b = 2 * k + 1 < N ? p[2 * k + 1] : 0.f;
    swap32(a, b);
    q[k] = a + b;
  }
  float r[NB / 4];
#pragma unroll
  for (int k = 0; k < NB / 4; ++k) {  // xor 16
    float a = q[2 * k], b = q[2 * k + 1];
    swap16(a, b);
    r[k] = a + b;
  }
  float v;
  if (NB == 8) {  // xor 8: lanes with bit 3 clear keep r[0], set keep r[NB / 4 - 1]
    const bool hi = (lane & 8) != 0;
    const float keep = hi ? r[NB / 4 - 1] : r[0], give = hi ? r[0] : r[NB / 4 - 1];
    v = keep + dpp_f<0x128>(give);  // row_ror:8 (a lane 8 apart: the other bit-3 half)
  } else {
    v = r[0] + dpp_f<0x128>(r[0]);
  }
  v += dpp_f<0xb1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4e>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror: the other quad of the 8
  return v;
}

// batch_grad over batch_dots' layout: lane L evaluates target batch_target(L)
// (its code fetched with one permute); counts the batch's non-finite scores.
template <int N, bool HSF>
__device__ __forceinline__ float batch_grad_l(float fl, int T, int code_l, int c0, float alpha, int lane,
                                              unsigned long long* stats) {
  const int t = batch_target<N>(lane);
  const int cl = __shfl(code_l, (c0 + t) & (kWave - 1));
  if (stats) {
    constexpr int grp = kBatchN<N> == 8 ? 7 : 15;
    const unsigned long long bad = ballot(t < T && (lane & grp) == 0 && !__builtin_isfinite(fl));
    if (bad && lane == 0) atomicAdd(stats + kNonFinite, (unsigned long long)__popcll(bad));
  }
  return grad_of<HSF>(fl, cl, alpha);
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// A batch of N > 8 targets (the deep HS pipeline of the low-occupancy
// kernel, train_epoch_deep_kernel) in groups of 8: group h's dots are folded
// and evaluated exactly as a batch of 8 would be (batch_dots / batch_grad_l),
// so each target's sum, sigma and g are the bits a batch of <= 8 gives. For N
// <= 8 this is the single batch_dots + batch_grad_l of before.
template <int N>
constexpr int kGroups = (N + 7) / 8;
template <int N>
constexpr int kGroupN = N < 8 ? N : 8;
template <int N, bool HSF>
__device__ __forceinline__ void batch_g(const float (&pd)[N], int T, int code_l, int c0, float alpha, int lane,
                                        unsigned long long* stats, float (&gl)[kGroups<N>]) {
  constexpr int G = kGroupN<N>;
#pragma unroll
  for (int h = 0; h < kGroups<N>; ++h) {
    float q[G];
#pragma unroll
    for (int t = 0; t < G; ++t) q[t] = (8 * h + t < N) ? pd[8 * h + t] : 0.f;
    gl[h] = batch_grad_l<G, HSF>(batch_dots<G>(q, lane), T - 8 * h, code_l, c0 + 8 * h, alpha, lane, stats);
  }
}
// g of target t from batch_g's per-group lanes
template <int N>
__device__ __forceinline__ float batch_gt(const float (&gl)[kGroups<N>], int t) {
  return readlane_f(gl[t / 8], batch_lane<kGroupN<N>>(t % 8));
}

// ---------------------------------------------------------------------------
// The per-target update (Word2Vec.cpp:238-246 HS; :261-268 NS), for up to
// MAXT distinct rows at once. Lane (t0 + t) of row_l / code_l holds target t's
// row and code (HS: Huffman code; NS: 1 - label). Rows are gathered together,
// then updated in target order so grad accumulates in the reference's order.
// Rows in [hot_lo, hot_hi) take the atomic path.
// ---------------------------------------------------------------------------
template <int NV, int MAXT, bool HSF>
__device__ __forceinline__ void apply_targets(float* M, int64_t pitch, int d, int lane, int T, int row_l,
                                              int code_l, int t0, const float (&x)[NV], float (&g)[NV],
                                              float alpha, int64_t hot_lo, int64_t hot_hi, const PrivRows& pr,
                                              unsigned long long* stats) {
  float r[MAXT][NV];
  int rows[MAXT];
  bool hot[MAXT], priv[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    rows[t] = readlane_i(row_l, t0 + t);
    priv[t] = pr.has(rows[t]);
    hot[t] = !priv[t] && rows[t] >= hot_lo && rows[t] < hot_hi;
    if (t < T) load_row<NV>(M, rows[t], pitch, d, lane, hot[t] || priv[t], r[t]);
  }
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {  // privatised rows: global value + this workgroup's pending delta
    if (t < T && priv[t]) {
      priv_read<NV>(pr, rows[t], lane, r[t]);
    }
  }
#if W2V_BATCH_DOTS
  float pd[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    pd[t] = 0.f;
    if (t < T) {  // the first product starts the sum (0 + p would cost an add per target)
      pd[t] = r[t][0] * x[0];
#pragma unroll
      for (int v = 1; v < NV; ++v) pd[t] += r[t][v] * x[v];
    }
  }
  float g_l[kGroups<MAXT>];
  batch_g<MAXT, HSF>(pd, T, code_l, t0, alpha, lane, stats, g_l);
#else
  float f[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    f[t] = 0.f;
    if (t < T) {
      float p = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) p += r[t][v] * x[v];
      f[t] = wave_sum(p);
    }
  }
  const float g_l = batch_grad<MAXT, HSF>(f, T, code_l, t0, alpha, lane);
#endif
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    if (t < T) {
#if W2V_BATCH_DOTS
      const float gt = batch_gt<MAXT>(g_l, t);
#else
      if (stats) note_nonfinite(stats, !__builtin_isfinite(f[t]), lane);
      const float gt = readlane_f(g_l, t);
#endif
      float delta[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        g[v] += gt * r[t][v];  // grad uses the pre-update row (:244 / :266)
        delta[v] = gt * x[v];
      }
      if (priv[t]) {  // ds_add_f32 into the workgroup's delta; flushed after the center
        priv_add<NV>(pr, rows[t], d, lane, delta);
      } else if (hot[t]) {
        if (!(W2V_EXP_SKIP & 1)) atomic_add_row<NV>(M, rows[t], pitch, d, lane, delta);
      } else {
#pragma unroll
        for (int v = 0; v < NV; ++v) r[t][v] += delta[v];
        if (!(W2V_EXP_SKIP & 64)) store_row<NV>(M, rows[t], pitch, d, lane, r[t]);
      }
    }
  }
}

// Move the workgroup's pending deltas of the dirty privatised rows into HBM
// (memory-side float atomics). The dirty mask and every delta word are taken
// with atomic swaps, so an add racing the flush from another wave of the
// workgroup is neither lost nor flushed twice (its dirty bit is set after its
// adds and survives until the next flush).
//
// Scale: a row that n workgroups update within one flush interval receives
// the mean of their deltas scaled to at most priv_avg concurrent
// contributions (local SGD on the few rows every wave updates; without it
// ~10^4 concurrent stale updates of those rows diverge). n is the expected
// count, computed on the host from the corpus statistics (launch_train:
// n = workgroups x P(a workgroup touches the row in flush_every centers)), so
// the scale is a fixed function of the row's frequency rank, not of the
// schedule (a.priv_sc / a.ctx_sc; 1 when priv_avg == 0).
template <int NV>
__device__ __forceinline__ void flush_private(const TrainArgs& a, const PrivRows& pr, int lane) {
  if (pr.n == 0) return;
  unsigned long long mw[2] = {0ull, 0ull};
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    unsigned long long m = 0;
    if (lane == 0 && 64 * w < pr.n) m = atomicExch(pr.dirty + w, 0ull);
    mw[w] = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(m >> 32)) << 32) |
            (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)m);
  }
  for (int w = 0; w < 2; ++w)
  for (unsigned long long m = mw[w]; m;) {
    const int p = 64 * w + __builtin_ctzll(m);
    m &= m - 1;
    const float sc = pr.ctx ? a.ctx_sc[p & (kCtxMax - 1)] : a.priv_sc[p];
    float* q = pr.delta + p * (NV * kWave) + lane;
    float* dst = pr.M + (pr.lo + p) * a.pitch + lane;
    if (W2V_PRIV_ADD == 2) {  // take the row under its lock (priv_add)
      float val[NV];
      priv_lock(pr, p, lane);
#pragma unroll
      for (int v = 0; v < NV; ++v) val[v] = q[kWave * v];
#pragma unroll
      for (int v = 0; v < NV; ++v) q[kWave * v] = 0.0f;
      priv_unlock(pr, p, lane);
#pragma unroll
      for (int v = 0; v < NV; ++v)
        if (val[v] != 0.0f && !(W2V_EXP_SKIP & 2))  // 0 past word_dim: skipped
          (void)__hip_atomic_fetch_add(dst + kWave * v, val[v] * sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const float val = atomicExch(q + kWave * v, 0.0f);  // 0 past word_dim: skipped
      if (val != 0.0f && !(W2V_EXP_SKIP & 2))
        (void)__hip_atomic_fetch_add(dst + kWave * v, val * sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// HS on the path of `word` (synapses1 rows), software-pipelined: the path's
// nodes are known up front and distinct, so batch b + 1's rows are gathered
// BEFORE batch b's updates are issued. vmcnt retires in order on gfx950, so a
// gather issued after a batch's stores and memory-side atomics would wait for
// all of them (~3000 cycles per atomic with every CU issuing); issued before
// them it waits only for its own loads. Same arithmetic, same order of the
// gradient sum as apply_targets (target order), so the sequential schedule
// stays bit-exact.
template <int NV, int MT>
__device__ __forceinline__ void hs_gather(const TrainArgs& a, int T, int row_l, int t0, const PrivRows& pr, int lane,
                                          float (&r)[MT][NV]) {
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    if (t < T) {
      const int row = readlane_i(row_l, t0 + t);
      load_row<NV>(a.S, row, a.pitch, a.dim, lane, pr.has(row) || row >= a.hot_s, r[t]);
    }
  }
}

// Scores of a gathered batch: privatised rows get the pending delta, then
// g += gt * row (pre-update row, :244) in target order; returns gt per target.
template <int NV, int MT>
__device__ __forceinline__ void hs_score(const TrainArgs& a, int T, int row_l, int code_l, int t0, const PrivRows& pr,
                                         int lane, const float (&x)[NV], float (&g)[NV], float alpha,
                                         float (&r)[MT][NV], float (&gt)[MT]) {
#pragma unroll
  for (int t = 0; t < MT; ++t)
    if (t < T) {
      const int row = readlane_i(row_l, t0 + t);
      if (pr.has(row)) priv_read<NV>(pr, row, lane, r[t]);
    }
#if W2V_BATCH_DOTS
  float pd[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    pd[t] = 0.f;
    if (t < T) {  // the first product starts the sum (0 + p would cost an add per target)
      pd[t] = r[t][0] * x[0];
#pragma unroll
      for (int v = 1; v < NV; ++v) pd[t] += r[t][v] * x[v];
    }
  }
  float g_l[kGroups<MT>];
  batch_g<MT, true>(pd, T, code_l, t0, alpha, lane, a.stats, g_l);
#else
  float f[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    f[t] = 0.f;
    if (t < T) {
      float p = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) p += r[t][v] * x[v];
      f[t] = wave_sum(p);
    }
  }
  const float g_l = batch_grad<MT, true>(f, T, code_l, t0, alpha, lane);
#endif
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    gt[t] = 0.f;
    if (t < T) {
#if W2V_BATCH_DOTS
      gt[t] = batch_gt<MT>(g_l, t);
#else
      note_nonfinite(a.stats, !__builtin_isfinite(f[t]), lane);
      gt[t] = readlane_f(g_l, t);
#endif
#pragma unroll
      for (int v = 0; v < NV; ++v) g[v] += gt[t] * r[t][v];
    }
  }
}

// The updates of a scored batch: LDS delta (privatised), memory-side atomic
// (hot), or the updated row stored (Hogwild).
template <int NV, int MT>
__device__ __forceinline__ void hs_apply(const TrainArgs& a, int T, int row_l, int t0, const PrivRows& pr, int lane,
                                         const float (&x)[NV], float (&r)[MT][NV], const float (&gt)[MT]) {
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    if (t < T) {
      const int row = readlane_i(row_l, t0 + t);
      float delta[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) delta[v] = gt[t] * x[v];
      if (pr.has(row)) {
        priv_add<NV>(pr, row, a.dim, lane, delta);
      } else if (row >= a.hot_s) {
        if (a.hot_sc) {  // damped to the hot-node average (wave-uniform row: one scalar load)
          const float s = a.hot_sc[row - a.hot_s];
#pragma unroll
          for (int v = 0; v < NV; ++v) delta[v] *= s;
        }
        if (!(W2V_EXP_SKIP & 1)) atomic_add_row<NV>(a.S, row, a.pitch, a.dim, lane, delta);
      } else {
#pragma unroll
        for (int v = 0; v < NV; ++v) r[t][v] += delta[v];
        if (!(W2V_EXP_SKIP & 64)) store_row<NV>(a.S, row, a.pitch, a.dim, lane, r[t]);
      }
    }
  }
}

template <int NV, int MAXT>
__device__ __forceinline__ void hs_word(const TrainArgs& a, int word, int lane, const float (&x)[NV],
                                        float (&g)[NV], float alpha, Counters& cnt, float* lds) {
#ifndef W2V_HS_MT
  constexpr int MT = MAXT / 2 > 0 ? MAXT / 2 : 1;  // two buffers of MT rows: the same registers as one of MAXT
#else  // experiments (tools/r03): rows per pipelined batch
  constexpr int MT = W2V_HS_MT;
#endif
  const PrivRows pr = (a.priv_M == a.S) ? out_rows<NV>(a, lds) : PrivRows();
  const int64_t cb = a.coff[word];
  const int L = (int)(a.coff[word + 1] - cb);
  for (int c0 = 0; c0 < L; c0 += kWave) {
    const int rem = min(kWave, L - c0);
    const int pt_l = (lane < rem) ? a.points[cb + c0 + lane] : 0;
    const int cd_l = (lane < rem) ? (int)a.codes[cb + c0 + lane] : 0;
    float ra[MT][NV], rb[MT][NV], gt[MT];
    if (a.strict) drain_vmem();
    hs_gather<NV, MT>(a, min(MT, rem), pt_l, 0, pr, lane, ra);
    for (int t0 = 0; t0 < rem; t0 += 2 * MT) {
      const int Ta = min(MT, rem - t0), Tb = min(MT, rem - t0 - MT);  // Tb <= 0: no second batch
      hs_score<NV, MT>(a, Ta, pt_l, cd_l, t0, pr, lane, x, g, alpha, ra, gt);
      if (Tb > 0) hs_gather<NV, MT>(a, Tb, pt_l, t0 + MT, pr, lane, rb);
      hs_apply<NV, MT>(a, Ta, pt_l, t0, pr, lane, x, ra, gt);
      if (Tb > 0) {
        hs_score<NV, MT>(a, Tb, pt_l, cd_l, t0 + MT, pr, lane, x, g, alpha, rb, gt);
        const int Tn = min(MT, rem - t0 - 2 * MT);
        if (Tn > 0) hs_gather<NV, MT>(a, Tn, pt_l, t0 + 2 * MT, pr, lane, ra);
        hs_apply<NV, MT>(a, Tb, pt_l, t0 + MT, pr, lane, x, rb, gt);
      }
    }
    cnt.targets += (unsigned long long)rem;
  }
}

// NS target list of positive `word` against `negw_l` lanes [base, base + neg):
// lane t of tgt_l holds target t (positive first, then first occurrences of
// the negatives that differ from it — the set semantics of
// Word2Vec.cpp:253-257); returns the count.
__device__ __forceinline__ int ns_targets(int neg, int word, int negw_l, int base, int lane, int& tgt_l) {
  const int nk = __shfl(negw_l, (base + lane) & (kWave - 1));
  bool dup = (lane >= neg) || (nk == word);
  for (int j = 0; j < neg - 1; ++j) {
    const int v = readlane_i(nk, j);
    dup = dup || (lane > j && nk == v);
  }
  const unsigned long long uniq = ballot(!dup);
  // compaction in one forward permute: the k-th unique draw (in lane order)
  // goes to lane 1 + k; duplicates to lane 0, which then takes the positive
  // (a walk over the set bits cost ~4 VALU + 6 SALU per target)
  const int k = __builtin_amdgcn_mbcnt_hi((unsigned)(uniq >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)uniq, 0u));
  const int v = __builtin_amdgcn_ds_permute((dup ? 0 : 1 + k) << 2, nk);
  tgt_l = (lane == 0) ? word : v;
  return 1 + __popcll(uniq);
}

// The T targets of tgt_l / code_l, MAXT rows per batch.
template <int NV, int MAXT>
__device__ __forceinline__ void apply_list(const TrainArgs& a, float* M, int T, int tgt_l, int code_l,
                                           const float (&x)[NV], float (&g)[NV], float alpha, Counters& cnt,
                                           const PrivRows& pr) {
  for (int t0 = 0; t0 < T; t0 += MAXT) {
    if (a.strict) drain_vmem();
    apply_targets<NV, MAXT, false>(M, a.pitch, a.dim, lane_id(), min(MAXT, T - t0), tgt_l, code_l, t0, x, g, alpha,
                                   0, a.hot_wc, pr, a.stats);
  }
  cnt.targets += (unsigned long long)T;
}

// Two consecutive contexts' NS updates as one batch (skip-gram, negative <=
// kPairNeg): context A's targets in slots [0, T1), context B's in [kPairHalf,
// kPairHalf + T2). All rows are gathered at once, so B's gathers no longer
// wait behind A's stores and memory-side atomics (vmcnt retires in order).
// The reference applies A before B (Word2Vec.cpp:329-349): a B target that
// is also one of A's takes A's updated row from the registers — the same fp32
// `row + g * x` a re-read would return on the sequential schedule, so parity
// is unchanged — and A's gradient terms accumulate before B's.
constexpr int kPairHalf = 6;
constexpr int kPairNeg = kPairHalf - 1;
#ifndef W2V_NS_PAIR  // 1: two contexts per batch (measured: no gain; off)
#define W2V_NS_PAIR 0
#endif
#ifndef W2V_NS_PAIR_MIN_NV
#define W2V_NS_PAIR_MIN_NV 3
#endif
template <int NV>
constexpr bool kNsPair = W2V_NS_PAIR && NV >= W2V_NS_PAIR_MIN_NV;  // d <= 128 keeps 64 VGPRs (8 waves/SIMD)

template <int NV>
__device__ __forceinline__ void pair_update(float* M, int64_t pitch, int d, int lane, int row, bool hot, bool priv,
                                            int code, float f, const float (&x)[NV], float (&g)[NV], float alpha,
                                            float (&r)[NV], const PrivRows& pr, unsigned long long* stats) {
  note_nonfinite(stats, !__builtin_isfinite(f), lane);
  const float e = expf(-f);
  const float s = ns_sigmoid(e);
  const float gt = ((float)(1 - code) - s) * alpha;
  float delta[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    g[v] += gt * r[v];  // grad uses the pre-update row (:266)
    delta[v] = gt * x[v];
    r[v] += delta[v];   // the updated row, for a later target of the other context
  }
  if (priv) {
    priv_add<NV>(pr, row, d, lane, delta);
  } else if (hot) {
    if (!(W2V_EXP_SKIP & 1)) atomic_add_row<NV>(M, row, pitch, d, lane, delta);
  } else {
    store_row<NV>(M, row, pitch, d, lane, r);
  }
}

template <int NV>
__device__ __forceinline__ void apply_pair(const TrainArgs& a, float* M, int T1, int T2, int row_l, int lane,
                                           const float (&x)[NV], float (&g)[NV], float alpha, const PrivRows& pr) {
  constexpr int H = kPairHalf, MP = 2 * kPairHalf;
  float r[MP][NV];
  int rows[MP];
  bool hot[MP], priv[MP], use[MP];
#pragma unroll
  for (int t = 0; t < MP; ++t) {
    use[t] = t < H ? t < T1 : t - H < T2;
    rows[t] = readlane_i(row_l, t);
    priv[t] = pr.has(rows[t]);
    hot[t] = !priv[t] && rows[t] < a.hot_wc;
    if (use[t]) load_row<NV>(M, rows[t], a.pitch, a.dim, lane, hot[t] || priv[t], r[t]);
  }
#pragma unroll
  for (int t = 0; t < MP; ++t)
    if (use[t] && priv[t]) priv_read<NV>(pr, rows[t], lane, r[t]);
  // context A: every score from the gathered rows, then the updates in target order
  float f[MP];
#pragma unroll
  for (int t = 0; t < H; ++t) {
    f[t] = 0.f;
    if (use[t]) {
      float p = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) p += r[t][v] * x[v];
      f[t] = wave_sum(p);
    }
  }
#pragma unroll
  for (int t = 0; t < H; ++t)
    if (use[t]) pair_update<NV>(M, a.pitch, a.dim, lane, rows[t], hot[t], priv[t], t == 0 ? 0 : 1, f[t], x, g, alpha,
                                r[t], pr, a.stats);
  // context B: a row A updated continues from A's result (targets of one
  // context are distinct, so at most one A slot matches)
#pragma unroll
  for (int t = H; t < MP; ++t)
#pragma unroll
    for (int u = 0; u < H; ++u)
      if (use[t] && use[u] && rows[t] == rows[u]) {
#pragma unroll
        for (int v = 0; v < NV; ++v) r[t][v] = r[u][v];
      }
#pragma unroll
  for (int t = H; t < MP; ++t) {
    f[t] = 0.f;
    if (use[t]) {
      float p = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) p += r[t][v] * x[v];
      f[t] = wave_sum(p);
    }
  }
#pragma unroll
  for (int t = H; t < MP; ++t)
    if (use[t]) pair_update<NV>(M, a.pitch, a.dim, lane, rows[t], hot[t], priv[t], t == H ? 0 : 1, f[t], x, g, alpha,
                                r[t], pr, a.stats);
}

// NS with positive `word` against `negw_l` lanes [base, base + neg).
template <int NV, int MAXT>
__device__ __forceinline__ void ns_word(const TrainArgs& a, float* M, int word, int negw_l, int base, int lane,
                                        const float (&x)[NV], float (&g)[NV], float alpha, Counters& cnt,
                                        float* lds) {
  const PrivRows pr = (a.priv_M == M) ? out_rows<NV>(a, lds) : PrivRows();
  int tgt_l;
  const int T = ns_targets(a.negative, word, negw_l, base, lane, tgt_l);
  apply_list<NV, MAXT>(a, M, T, tgt_l, (lane == 0) ? 0 : 1, x, g, alpha, cnt, pr);
}

// ---------------------------------------------------------------------------
// NS with more draws than a wave has lanes (negative >= 64; the reference
// takes any value, Word2Vec.cpp:254-255). The targets keep the set semantics
// and the order of ns_targets — the positive, then the first occurrence of
// every negative that differs from it, in draw order — taken 64 draws at a
// time: chunk ch holds draws k = 64 ch + lane; a draw is a duplicate if an
// earlier draw of its chunk or any draw of an earlier chunk (drawn again: the
// same counter gives the same word) is the same word. Each chunk's new
// targets are applied before the next chunk's are found (a duplicate test
// needs only the words, not the rows).
// ---------------------------------------------------------------------------
#ifndef W2V_MANY_NEG  // timing experiments only: 0 compiles the path out (negative >= 64 then trains wrongly)
#define W2V_MANY_NEG 1
#endif
template <bool REPLAY>
__device__ __forceinline__ int draw_chunk(const TrainArgs& a, uint32_t s, uint32_t i, int slot, int ch, int lane,
                                          const uint32_t* rp) {
  const int k = kWave * ch + lane;
  int w = -1;
  if (k < a.negative) {
    const uint32_t pos = REPLAY ? rp[k] : philox_table_pos(a, s, i, (uint32_t)slot, (uint32_t)k);
    w = (int)a.table[pos];
  }
  return w;
}

template <int NV, int MAXT, bool REPLAY>
__device__ __forceinline__ void ns_word_many(const TrainArgs& a, float* M, int word, uint32_t s, uint32_t i, int slot,
                                          int lane, const float (&x)[NV], float (&g)[NV], float alpha,
                                          Counters& cnt, float* lds, const uint32_t*& rp) {
  const PrivRows pr = (a.priv_M == M) ? out_rows<NV>(a, lds) : PrivRows();
  const int neg = a.negative;
  const int nch = (neg + kWave - 1) / kWave;
  apply_list<NV, MAXT>(a, M, 1, word, 0, x, g, alpha, cnt, pr);  // the positive (label 1)
  for (int ch = 0; ch < nch; ++ch) {
    const int w = draw_chunk<REPLAY>(a, s, i, slot, ch, lane, rp);
    bool dup = (w < 0) || (w == word);
    for (int j = 0; j < kWave - 1; ++j) {
      const int v = readlane_i(w, j);
      dup = dup || (lane > j && v == w);
    }
    for (int c2 = 0; c2 < ch; ++c2) {
      const int wp = draw_chunk<REPLAY>(a, s, i, slot, c2, lane, rp);
      for (int j = 0; j < kWave; ++j) dup = dup || (readlane_i(wp, j) == w);
    }
    unsigned long long uniq = ballot(!dup);
    int tgt_l = 0, m = 0;
    while (uniq) {
      const int b = __builtin_ctzll(uniq);
      uniq &= uniq - 1;
      const int v = readlane_i(w, b);
      if (lane == m) tgt_l = v;
      ++m;
    }
    if (m > 0) apply_list<NV, MAXT>(a, M, m, tgt_l, 1, x, g, alpha, cnt, pr);  // negatives (label 0)
  }
  cnt.draws += (unsigned long long)neg;
  if (REPLAY) rp += neg;
}

// Draw table words for `ndraw` (slot, k) pairs starting at slot `slot0`:
// lane t -> slot0 + t / neg, k = t % neg.
template <bool REPLAY>
__device__ __forceinline__ int draw_negatives(const TrainArgs& a, uint32_t s, uint32_t i, int slot0, int ndraw,
                                              int lane, const uint32_t*& rp) {
  int w = 0;
  if (lane < ndraw) {
    uint32_t pos;
    if (REPLAY) {
      pos = rp[lane];
    } else {
      const int neg = a.negative;
      pos = philox_table_pos(a, s, i, (uint32_t)(slot0 + lane / neg), (uint32_t)(lane % neg));
    }
    w = (int)a.table[pos];
  }
  if (REPLAY) rp += ndraw;
  return w;
}

// ---------------------------------------------------------------------------
// Skip-gram center (Word2Vec.cpp:329-351) with its window [lo, hi).
// ---------------------------------------------------------------------------
template <int NV, int MAXT, bool HS, bool NS, bool REPLAY>
__device__ __forceinline__ void sg_center(const TrainArgs& a, float* lds, const int32_t* sent, int len, int i, int c, int rw,
                                          uint32_t s, float alpha, const uint32_t*& rp, Counters& cnt, int lane) {
  const int lo = max(0, i - a.window + rw), hi = min(len, i + a.window + 1 - rw);
  const int span = hi - lo;
  const bool hot_c = c < a.hot_wc;
  float x[NV], g[NV];
  if (a.strict) drain_vmem();
  load_row<NV>(a.W, c, a.pitch, a.dim, lane, hot_c, x);
#pragma unroll
  for (int v = 0; v < NV; ++v) g[v] = 0.f;
  const int ctx_l = (lane < span) ? sent[lo + lane] : 0;
  cnt.centers += 1;
  cnt.contexts += (unsigned long long)(span - 1);
  const int nctx = span - 1;
  const int neg = a.negative;
  if (NS && !HS && kNsPair<NV> && neg <= kPairNeg && span <= kWave) {
    // contexts two at a time (apply_pair); the table draws of G2 contexts at once
    const int me = i - lo;
    const int cw_l = sent[lo + min(lane + (lane >= me ? 1 : 0), span - 1)];  // lane k: the k-th context word
    const int G2 = max(2, (kWave / neg) & ~1);
    const PrivRows pr = (a.priv_M == a.C) ? out_rows<NV>(a, lds) : PrivRows();
    int negw_l = 0;
    for (int k = 0; k < nctx; k += 2) {
      const int gs = k % G2;
      if (gs == 0) {
        const int nd = min(G2, nctx - k) * neg;
        negw_l = draw_negatives<REPLAY>(a, s, (uint32_t)i, k, nd, lane, rp);
        cnt.draws += (unsigned long long)nd;
      }
      int ta = 0, tb = 0;
      const int T1 = ns_targets(neg, readlane_i(cw_l, k), negw_l, gs * neg, lane, ta);
      const int T2 = (k + 1 < nctx) ? ns_targets(neg, readlane_i(cw_l, k + 1), negw_l, (gs + 1) * neg, lane, tb) : 0;
      // every lane takes part in the permute: a lane whose exec bit is off
      // supplies no data to ds_bpermute, so a shuffle under `lane >= kPairHalf`
      // would read B's targets from switched-off lanes 0..5
      const int tb_s = __shfl(tb, (lane - kPairHalf) & (kWave - 1));
      const int tgt_l = lane < kPairHalf ? ta : tb_s;
      if (a.strict) drain_vmem();
      apply_pair<NV>(a, a.C, T1, T2, tgt_l, lane, x, g, alpha, pr);
      cnt.targets += (unsigned long long)(T1 + T2);
    }
    cnt.stamp(3);
    add_to_row<NV>(a.W, c, hot_c, a.pitch, a.dim, lane, g);  // W.row(center) += neu1_grad (:351)
    cnt.stamp(4);
    return;
  }
  const int G = NS ? max(1, kWave / max(neg, 1)) : 1;
  int negw_l = 0;
  int slot = 0;
  for (int j = lo; j < hi; ++j) {
    if (j == i) continue;
    const int w = (j - lo < kWave) ? readlane_i(ctx_l, j - lo) : uniform_i(sent[j]);  // window > 31: span > 64
    if (HS) hs_word<NV, MAXT>(a, w, lane, x, g, alpha, cnt, lds);
    if (W2V_MANY_NEG && NS && neg >= kWave) {
      ns_word_many<NV, MAXT, REPLAY>(a, a.C, w, s, (uint32_t)i, slot, lane, x, g, alpha, cnt, lds, rp);
    } else if (NS) {
      const int gs = slot % G;
      if (gs == 0) {
        const int nd = min(G, nctx - slot) * neg;
        negw_l = draw_negatives<REPLAY>(a, s, (uint32_t)i, slot, nd, lane, rp);
        cnt.draws += (unsigned long long)nd;
      }
      ns_word<NV, MAXT>(a, a.C, w, negw_l, gs * neg, lane, x, g, alpha, cnt, lds);
    }
    ++slot;
  }
  cnt.stamp(3);
  add_to_row<NV>(a.W, c, hot_c, a.pitch, a.dim, lane, g);  // W.row(center) += neu1_grad (:351)
  cnt.stamp(4);
}

// ---------------------------------------------------------------------------
// CBOW center (Word2Vec.cpp:286-315): the unique context ids in ascending
// order (std::set), then cbow_tail. row_of(r) is the r-th of them.
// ---------------------------------------------------------------------------
template <int NV, int MAXT, bool HS, bool NS, bool REPLAY, class RowOf>
__device__ __forceinline__ void cbow_tail(const TrainArgs& a, float* lds, int i, int c, int n, int U, RowOf row_of,
                                         uint32_t s, float alpha, const uint32_t*& rp, Counters& cnt, int lane) {
  cnt.centers += 1;
  cnt.contexts += (unsigned long long)U;
  float h[NV], g[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) h[v] = g[v] = 0.f;
  const PrivRows cx = ctx_rows<NV>(a, lds);  // the hottest context rows: global value + pending delta
  if (a.strict) drain_vmem();
  for (int r0 = 0; r0 < U; r0 += MAXT) {
    float rr[MAXT][NV];
#pragma unroll
    for (int t = 0; t < MAXT; ++t)
      if (r0 + t < U) {
        const int row = row_of(r0 + t);
        load_row<NV>(a.C, row, a.pitch, a.dim, lane, row < a.hot_wc || cx.has(row), rr[t]);
      }
#pragma unroll
    for (int t = 0; t < MAXT; ++t)
      if (r0 + t < U) {
        const int row = row_of(r0 + t);
        if (cx.has(row)) priv_read<NV>(cx, row, lane, rr[t]);
#pragma unroll
        for (int v = 0; v < NV; ++v) h[v] += rr[t][v];
      }
  }
  const float nf = (float)n;
  if (a.cbow_mean) {
#pragma unroll
    for (int v = 0; v < NV; ++v) h[v] /= nf;
  }
  cnt.stamp(2);
  if (HS) hs_word<NV, MAXT>(a, c, lane, h, g, alpha, cnt, lds);
  if (W2V_MANY_NEG && NS && a.negative >= kWave) {
    ns_word_many<NV, MAXT, REPLAY>(a, a.W, c, s, (uint32_t)i, 0, lane, h, g, alpha, cnt, lds, rp);
  } else if (NS) {
    const int nd = a.negative;
    const int negw_l = draw_negatives<REPLAY>(a, s, (uint32_t)i, 0, nd, lane, rp);
    cnt.draws += (unsigned long long)nd;
    ns_word<NV, MAXT>(a, a.W, c, negw_l, 0, lane, h, g, alpha, cnt, lds);
  }
  cnt.stamp(3);
  if (a.cbow_mean) {
#pragma unroll
    for (int v = 0; v < NV; ++v) g[v] /= nf;
  }
  // C.row(id) += neu1_grad for every unique id (:315). The plain (Hogwild)
  // rows of a batch are all gathered before any of them is stored: with
  // in-order vmcnt a row-by-row read-modify-write would make each gather wait
  // for the previous row's store.
  for (int r0 = 0; r0 < U; r0 += MAXT) {
    float cur[MAXT][NV];
#pragma unroll
    for (int t = 0; t < MAXT; ++t)
      if (r0 + t < U) {
        const int row = row_of(r0 + t);
        if (!cx.has(row) && row >= a.hot_wc) load_row<NV>(a.C, row, a.pitch, a.dim, lane, false, cur[t]);
      }
#pragma unroll
    for (int t = 0; t < MAXT; ++t)
      if (r0 + t < U) {
        const int row = row_of(r0 + t);
        if (cx.has(row)) {
          priv_add<NV>(cx, row, a.dim, lane, g);
        } else if (row < a.hot_wc) {
          if (!(W2V_EXP_SKIP & 4)) atomic_add_row<NV>(a.C, row, a.pitch, a.dim, lane, g);
        } else {
#pragma unroll
          for (int v = 0; v < NV; ++v) cur[t][v] += g[v];
          if (!(W2V_EXP_SKIP & 64)) store_row<NV>(a.C, row, a.pitch, a.dim, lane, cur[t]);
        }
      }
  }
  cnt.stamp(4);
}

template <int NV, int MAXT, bool HS, bool NS, bool REPLAY>
__device__ __forceinline__ void cbow_center(const TrainArgs& a, float* lds, const int32_t* sent, int len, int i, int c, int rw,
                                            uint32_t s, float alpha, const uint32_t*& rp, Counters& cnt, int lane) {
  const int lo = max(0, i - a.window + rw), hi = min(len, i + a.window + 1 - rw);
  const int n = hi - lo - 1;  // neu1_num, positional
  if (n <= 0) return;
  const int span = hi - lo;
  const int me = i - lo;
  const bool valid = lane < span && lane != me;
  const int id = valid ? sent[lo + lane] : 0;
  // std::set semantics: unique ids, visited in ascending order.
  bool dup = !valid;
  for (int j = 0; j < span; ++j) {
    const int v = readlane_i(id, j);
    dup = dup || (j != me && j < lane && v == id);
  }
  const unsigned long long uniq = ballot(!dup);
  const int U = __popcll(uniq);
  int rank = 0;
  {
    unsigned long long m = uniq;
    while (m) {
      const int b = __builtin_ctzll(m);
      m &= m - 1;
      rank += (readlane_i(id, b) < id) ? 1 : 0;
    }
  }
  int sid = 0;
  {
    unsigned long long m = uniq;
    while (m) {
      const int b = __builtin_ctzll(m);
      m &= m - 1;
      const int v = readlane_i(id, b), rk = readlane_i(rank, b);
      if (lane == rk) sid = v;
    }
  }
  cnt.stamp(1);
  cbow_tail<NV, MAXT, HS, NS, REPLAY>(a, lds, i, c, n, U, [&](int r) { return readlane_i(sid, r); }, s, alpha, rp,
                                      cnt, lane);
}

// Lane-register arrays of NCH x 64 positions: element j is lane j % 64 of register j / 64.
template <int NCH>
__device__ __forceinline__ int pick_lane(const int (&v)[NCH], int j) {
  int r = 0;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch)
    if (ch == (j >> 6)) r = readlane_i(v[ch], j & (kWave - 1));
  return r;
}

// CBOW center for windows wider than a wave (2 * window + 1 > 64, window <=
// 32 * NCH - 1): the same set semantics and visiting order as cbow_center, the
// span's positions held NCH per lane (position lo + 64 ch + lane).
template <int NV, int MAXT, bool HS, bool NS, bool REPLAY, int NCH>
__device__ __forceinline__ void cbow_center_wide(const TrainArgs& a, float* lds, const int32_t* sent, int len, int i,
                                                 int c, int rw, uint32_t s, float alpha, const uint32_t*& rp,
                                                 Counters& cnt, int lane) {
  const int lo = max(0, i - a.window + rw), hi = min(len, i + a.window + 1 - rw);
  const int n = hi - lo - 1;
  if (n <= 0) return;
  const int span = hi - lo;
  const int me = i - lo;
  int id[NCH];
  bool dup[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int p = kWave * ch + lane;
    const bool valid = p < span && p != me;
    id[ch] = valid ? sent[lo + p] : 0;
    dup[ch] = !valid;
  }
  for (int j = 0; j < span; ++j) {  // a later position repeating an earlier valid id is a duplicate
    if (j == me) continue;
    const int v = pick_lane<NCH>(id, j);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) dup[ch] = dup[ch] || (j < kWave * ch + lane && v == id[ch]);
  }
  unsigned long long uq[NCH];
  int U = 0;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    uq[ch] = ballot(!dup[ch]);
    U += __popcll(uq[ch]);
  }
  int rank[NCH], sid[NCH];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) rank[ch] = sid[ch] = 0;
#pragma unroll
  for (int c2 = 0; c2 < NCH; ++c2) {
    unsigned long long m = uq[c2];
    while (m) {
      const int b = __builtin_ctzll(m);
      m &= m - 1;
      const int v = readlane_i(id[c2], b);
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) rank[ch] += (v < id[ch]) ? 1 : 0;
    }
  }
#pragma unroll
  for (int c2 = 0; c2 < NCH; ++c2) {
    unsigned long long m = uq[c2];
    while (m) {
      const int b = __builtin_ctzll(m);
      m &= m - 1;
      const int v = readlane_i(id[c2], b), rk = readlane_i(rank[c2], b);
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch)
        if (ch == (rk >> 6) && lane == (rk & (kWave - 1))) sid[ch] = v;
    }
  }
  cbow_tail<NV, MAXT, HS, NS, REPLAY>(a, lds, i, c, n, U, [&](int r) { return pick_lane<NCH>(sid, r); }, s, alpha,
                                      rp, cnt, lane);
}

constexpr int kWideChunks = 4;  // wide-window CBOW kernels: window <= 32 * kWideChunks - 1 in registers
constexpr int kMaxWideWindow = 32 * kWideChunks - 1;
// Any larger window (the reference takes any, Word2Vec.cpp:285): cbow_center_huge.
constexpr int kMaxWindow = (1 << 20) - 1;
// Ints of a wave's cbow_center_huge scratch slice for `window`: the unique
// ids (<= 2 window) and one 64-bit unique mask per 64 span positions.
__host__ __device__ inline int64_t huge_stride(int window) {
  const int64_t span = 2 * (int64_t)window + 1;
  return 2 * (int64_t)window + 2 * ((span + 63) / 64) + 2;
}

// CBOW center for windows past kMaxWideWindow: the same set semantics and
// ascending visiting order as cbow_center, with the span read from the
// sentence 64 positions at a time. Pass 1 marks each position that is not a
// repeat of an earlier valid one (a scalar walk over the earlier positions)
// and keeps each chunk's unique mask in this wave's slice of a global scratch;
// pass 2 ranks every unique id among all of them (the count of smaller ones)
// and writes it to slot `rank`, so the slice holds the ids in ascending order
// for cbow_tail. O(span^2 / 64) scalar steps per center: the price of a window
// no register set holds.
template <int NV, int MAXT, bool HS, bool NS, bool REPLAY>
__device__ __forceinline__ void cbow_center_huge(const TrainArgs& a, float* lds, const int32_t* sent, int len, int i,
                                                 int c, int rw, uint32_t s, float alpha, const uint32_t*& rp,
                                                 Counters& cnt, int lane) {
  const int lo = max(0, i - a.window + rw), hi = min(len, i + a.window + 1 - rw);
  const int n = hi - lo - 1;
  if (n <= 0) return;
  const int span = hi - lo;
  const int me = i - lo;
  const int nch = (span + kWave - 1) / kWave;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  int32_t* ids_out = a.wide_ids + wave * a.wide_stride;
  int32_t* masks = ids_out + 2 * (int64_t)a.window;  // 2 ints per chunk
  int U = 0;
  for (int ch = 0; ch < nch; ++ch) {
    const int p = kWave * ch + lane;
    const bool valid = p < span && p != me;
    const int id = valid ? sent[lo + p] : -1;
    bool dup = !valid;
    const int jmax = min(span, kWave * ch + kWave - 1);
    for (int j = 0; j < jmax; ++j) {
      if (j == me) continue;
      const int v = uniform_i(sent[lo + j]);
      dup = dup || (j < p && v == id);
    }
    const unsigned long long uq = ballot(!dup);
    U += __popcll(uq);
    if (lane == 0) {
      masks[2 * ch] = (int32_t)(uint32_t)uq;
      masks[2 * ch + 1] = (int32_t)(uint32_t)(uq >> 32);
    }
  }
  drain_vmem();
  for (int ch = 0; ch < nch; ++ch) {
    const int p = kWave * ch + lane;
    const int id = (p < span) ? sent[lo + p] : -1;
    const unsigned long long mine =
        ((unsigned long long)(uint32_t)__hip_atomic_load(masks + 2 * ch + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) << 32) |
        (uint32_t)__hip_atomic_load(masks + 2 * ch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool uniq = (mine >> lane) & 1ull;
    int rank = 0;
    for (int c2 = 0; c2 < nch; ++c2) {
      unsigned long long m =
          ((unsigned long long)(uint32_t)__hip_atomic_load(masks + 2 * c2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) << 32) |
          (uint32_t)__hip_atomic_load(masks + 2 * c2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      m = ((unsigned long long)(uint32_t)readlane_i((int)(m >> 32), 0) << 32) | (uint32_t)readlane_i((int)(uint32_t)m, 0);
      while (m) {
        const int b = __builtin_ctzll(m);
        m &= m - 1;
        rank += (uniform_i(sent[lo + kWave * c2 + b]) < id) ? 1 : 0;
      }
    }
    if (uniq) ids_out[rank] = id;
  }
  drain_vmem();
  cbow_tail<NV, MAXT, HS, NS, REPLAY>(
      a, lds, i, c, n, U,
      [&](int r) { return uniform_i(__hip_atomic_load(ids_out + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)); },
      s, alpha, rp, cnt, lane);
}

template <int NV, int MAXT, bool CBOW, bool HS, bool NS, bool REPLAY, bool WIDE>
__device__ __forceinline__ void center(const TrainArgs& a, float* lds, const int32_t* sent, int len, int i, int c,
                                       int rw, uint32_t s, float alpha, const uint32_t*& rp, Counters& cnt,
                                       int lane) {
  cnt.stamp(0);
  if (CBOW && WIDE && a.window > kMaxWideWindow)
    cbow_center_huge<NV, MAXT, HS, NS, REPLAY>(a, lds, sent, len, i, c, rw, s, alpha, rp, cnt, lane);
  else if (CBOW && WIDE)
    cbow_center_wide<NV, MAXT, HS, NS, REPLAY, kWideChunks>(a, lds, sent, len, i, c, rw, s, alpha, rp, cnt, lane);
  else if (CBOW)
    cbow_center<NV, MAXT, HS, NS, REPLAY>(a, lds, sent, len, i, c, rw, s, alpha, rp, cnt, lane);
  else
    sg_center<NV, MAXT, HS, NS, REPLAY>(a, lds, sent, len, i, c, rw, s, alpha, rp, cnt, lane);
  if (lds != nullptr) {
    // Bounded staleness with aggregation: the workgroup's waves share one
    // center count, and the wave that completes every flush_every-th center
    // drains the deltas all of them accumulated (one atomic per dirty row
    // instead of one per update and wave).
    unsigned* done = reinterpret_cast<unsigned*>(lds) + 8;
    unsigned n = 0;
    if (lane == 0) n = atomicAdd(done, 1u) + 1u;
    n = (unsigned)__builtin_amdgcn_readfirstlane((int)n);
    cnt.stamp(7);
    if (a.priv_n > 0 && n % (unsigned)a.flush_every == 0u) flush_private<NV>(a, out_rows<NV>(a, lds), lane);
    cnt.stamp(5);
    if (a.ctx_n > 0 && n % (unsigned)a.ctx_flush_every == 0u) flush_private<NV>(a, ctx_rows<NV>(a, lds), lane);
    cnt.stamp(6);
  }
}

// ---------------------------------------------------------------------------
// The epoch kernel: wavefronts dequeue sentences (Word2Vec.cpp:375-394).
// ---------------------------------------------------------------------------
template <int NV, int MAXT, bool CBOW, bool HS, bool NS, bool REPLAY, bool WIDE>
__device__ __forceinline__ void train_epoch(const TrainArgs& a) {
  extern __shared__ float w2v_lds[];
  const int lane = lane_id();
  float* lds = (a.priv_n + a.ctx_n) > 0 ? w2v_lds : nullptr;
  if (lds) {
    const int64_t words = lds_header_words(a.priv_n, a.ctx_n) + (int64_t)(a.priv_n + a.ctx_n) * (NV * kWave);
    for (int64_t k = threadIdx.x; k < words; k += blockDim.x) lds[k] = 0.0f;
    __syncthreads();
  }
  Counters cnt;
#ifdef W2V_PP_PROF
  cnt.t = __builtin_amdgcn_s_memtime();
#endif
  float alpha = a.init_alpha;
  bool first = true;
  const uint32_t wmax = (uint32_t)(a.window < 1 ? 1 : a.window);
  // A work item is one sentence, or (nseg > 1: parallel Philox schedule) one
  // seg_len-token segment of it, so that the last round of a launch is short
  // (a few thousand waves, ~1000-token sentences: whole-sentence items leave
  // most waves idle while the last sentences finish). Segment g of a sentence
  // trains the centers [g * seg_len, (g + 1) * seg_len) with the whole sentence
  // as their windows, exactly what the whole-sentence wave does for them.
  const uint32_t nseg = (uint32_t)(a.nseg > 1 ? a.nseg : 1);
  const int64_t n_items = a.n_sent * (int64_t)nseg;
  for (;;) {
    uint32_t kk = 0;
    if (lane == 0) kk = atomicAdd(a.work, 1u);
    kk = (uint32_t)uniform_i((int)kk);
    if ((int64_t)kk >= n_items) break;
    const uint32_t k = kk / nseg, seg = kk - k * nseg;
    const int64_t s = a.order ? a.order[k] : (int64_t)k;
    if (s < 0 || s >= a.n_corpus) continue;  // a caller-supplied device order is not host-checked
    if (a.fixed_alpha > 0.0f) {
      alpha = a.fixed_alpha;
    } else if (first || (k % 10u) == 0u) {
      const unsigned long long cw = __hip_atomic_load(a.words, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const float al = (float)(a.init_alpha * (1.0 - 1.0 / a.iter * (double)cw / a.train_words));
      alpha = (a.min_alpha < al) ? al : a.min_alpha;
      first = false;
    }
    const int64_t base = a.soff[s];
    const int len = (int)(a.soff[s + 1] - base);
    const int32_t* sent = a.ids + base;
    const uint32_t* rp = nullptr;
    if (REPLAY) {
      rp = a.replay + a.replay_off[s];
      for (int i = 0; i < len; ++i) {
        const int c = sent[i];
        const float u = __int_as_float((int)rp[0]);
        ++rp;
        if (a.keep[c] < u) continue;
        const int rw = (int)rp[0];
        ++rp;
        center<NV, MAXT, CBOW, HS, NS, REPLAY, WIDE>(a, lds, sent, len, i, c, rw, (uint32_t)s, alpha, rp, cnt, lane);
      }
    } else {
      const int seg_lo = nseg > 1 ? min(len, (int)seg * a.seg_len) : 0;
      const int seg_hi = nseg > 1 ? min(len, seg_lo + a.seg_len) : len;
      for (int i0 = seg_lo; i0 < seg_hi; i0 += kWave) {
        const int ii = i0 + lane;
        const bool in = ii < seg_hi;
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
          const int c = readlane_i(c_l, b), rw = readlane_i(rw_l, b);
          center<NV, MAXT, CBOW, HS, NS, REPLAY, WIDE>(a, lds, sent, len, i0 + b, c, rw, (uint32_t)s, alpha, rp,
                                                        cnt, lane);
        }
      }
    }
    if (REPLAY || nseg == 1) {
      if (lane == 0) atomicAdd(a.words, (unsigned long long)len);
      cnt.sentences += 1;
    } else {
      const int seg_lo = min(len, (int)seg * a.seg_len), seg_hi = min(len, seg_lo + a.seg_len);
      if (lane == 0 && seg_hi > seg_lo) atomicAdd(a.words, (unsigned long long)(seg_hi - seg_lo));
      cnt.sentences += (seg == 0) ? 1 : 0;
    }
  }
  flush_private<NV>(a, out_rows<NV>(a, lds), lane);
  flush_private<NV>(a, ctx_rows<NV>(a, lds), lane);
#ifdef W2V_PP_PROF
  cnt.stamp(0);
  if (lane == 0 && (threadIdx.x / kWave) % 4 == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2))
    printf("PPPROF block %u wave %d centers %llu: %llu %llu %llu %llu %llu %llu %llu %llu\n", blockIdx.x,
           (int)(threadIdx.x / kWave), cnt.centers, cnt.acc[0], cnt.acc[1], cnt.acc[2], cnt.acc[3], cnt.acc[4],
           cnt.acc[5], cnt.acc[6], cnt.acc[7]);
#endif
  if (lane == 0) {
    atomicAdd(&a.stats[0], cnt.centers);
    atomicAdd(&a.stats[1], cnt.contexts);
    atomicAdd(&a.stats[2], cnt.targets);
    atomicAdd(&a.stats[3], cnt.draws);
    atomicAdd(&a.stats[4], cnt.sentences);
  }
}

template <int NV, int MAXT, bool CBOW, bool HS, bool NS, bool REPLAY, bool WIDE>
__global__ __launch_bounds__(kMaxBlock<NV>, kMinWaves<NV>) void train_epoch_kernel(TrainArgs a) {
  train_epoch<NV, MAXT, CBOW, HS, NS, REPLAY, WIDE>(a);
}

// The same epoch for a launch that runs few waves (round 6: large-vocabulary
// HS capped at kHsRootPressure root updates in flight, 1-6 waves per CU):
// workgroups of <= 4 waves and a 256-VGPR budget (2 waves per SIMD), so a
// Huffman path is gathered kDeepMaxT / 2 nodes at a time instead of 4 —
// a wave that has the CU to itself is latency-bound on its path's round
// trips. Same arithmetic in the same order as train_epoch_kernel.
template <int NV>
constexpr int kDeepMaxT = NV <= 2 ? 32 : NV <= 4 ? 24 : NV <= 6 ? 16 : NV <= 16 ? 8 : 4;
constexpr int kDeepBlock = 256;
template <int NV, int MAXT, bool CBOW, bool HS, bool NS, bool REPLAY, bool WIDE>
__global__ __launch_bounds__(kDeepBlock, 2) void train_epoch_deep_kernel(TrainArgs a) {
  train_epoch<NV, MAXT, CBOW, HS, NS, REPLAY, WIDE>(a);
}

// Sequential target updates for w2v_dev_apply_rows (one wave): target t is
// row t of M, applied in order (rows are distinct; plain read-modify-write).
template <int NV>
__global__ __launch_bounds__(64) void apply_rows_kernel(float* M, int64_t pitch, int d, const float* x_in,
                                                        float* grad_io, const uint8_t* codes, int n, float alpha,
                                                        int hs_form) {
  const int lane = lane_id();
  float x[NV], g[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int e = lane + kWave * v;
    x[v] = (e < d) ? x_in[e] : 0.f;
    g[v] = (e < d) ? grad_io[e] : 0.f;
  }
  for (int t = 0; t < n; ++t) {
    const int code = (int)codes[t];
    if (hs_form)
      apply_targets<NV, 1, true>(M, pitch, d, lane, 1, t, code, 0, x, g, alpha, 0, 0, PrivRows(), nullptr);
    else
      apply_targets<NV, 1, false>(M, pitch, d, lane, 1, t, code, 0, x, g, alpha, 0, 0, PrivRows(), nullptr);
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int e = lane + kWave * v;
    if (e < d) grad_io[e] = g[v];
  }
}

}  // namespace w2v
