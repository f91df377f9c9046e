// w2v_group.hip — multi-GPU data parallelism behind the C-ABI (include/w2v_dev.h,
// w2v_group_*): model replicas synchronised with RCCL over xGMI.
//
// The reference parallelises only with OpenMP threads sharing ONE model
// (Word2Vec.cpp:375-394): every thread's update lands in the shared rows. Across
// GPUs every device trains a full replica of W / C / synapses1 on its shard of
// the sentences (the Hogwild kernels), and at the end of every round the
// replicas exchange what they learned:
//   D_i = M_i - P            (replica i's updates since the last exchange; P =
//                             the shared model then, identical on every replica)
//   A   = sum_i D_i          (one ncclAllReduce per matrix over xGMI)
//   M_i <- P + A / c, P <- M_i
// with c per row. W2V_GROUP_ADAPTIVE: c = the row's coherence |sum D|^2 /
// sum |D|^2 (at least 1): the mean of the replicas' moves of a row they all
// moved the same way (a frequent row each replica drives to the same optimum:
// summing R such moves overshoots R-fold and diverges), the sum of
// independent moves (a rare row each replica saw a different part of).
// W2V_GROUP_SPLIT: c = R for the rows a replica is expected to update at
// least `saturated_updates` times per round (from the corpus statistics: such
// a row reaches its local optimum within the round in every replica, and the
// sum of R such moves overshoots R-fold), c = 1 for the rest (small,
// independent moves that one model would have made one after another).
// W2V_GROUP_SUM: c = 1 — every update counts once,
// as in the reference's one shared model; the replicas are Hogwild threads
// whose writes become visible to each other at the round boundary.
// W2V_GROUP_ROW_AVERAGE: c = the number of replicas whose round changed the
// row. W2V_GROUP_AVERAGE: c = R (plain model averaging).
// What the exchange does to quality is the algorithm's, not the
// implementation's: a CPU simulation with the sequential oracle per replica
//  reproduces the GPU scores, and summing is the only mode that
// converges to the single-model result as rounds shorten (2 replicas on a 2 M
// token corpus, analogy at 1 / 4 / 16 / 32 / 64 rounds per epoch: 11 / 22 /
// 50 / 64 / 68 against 66 for one model; averaging: 10 at 4 and 15 at 16
// rounds). The replicas must exchange often relative to how fast the rows
// move; with more replicas, more often.
// Each matrix is one contiguous V x pitch fp32 buffer, the message size RCCL's
// rings over the seven xGMI links run at full rate, issued as one group over
// all matrices and all replicas this process drives.
//
// Overlap (w2v_group_set_overlap): the all-reduce of round r's deltas runs on a
// communication stream while round r + 1 trains; at the next boundary the
// training stream extracts round r + 1's delta and folds in the pending sum
// (M += s A - D_r: the others' round-r updates; its own are already in M).
// The exchange is then delayed by one round — the double-buffered replicas of
// SURVEY.md §8(e).
//
// Replicas on ONE device (several handles on the same GPU, e.g. to rehearse a
// multi-GPU run on one card) cannot join one RCCL communicator; their deltas
// are summed by a kernel reading every replica's buffer directly.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "w2v_dev.h"
#include "w2v_dev_internal.hpp"

namespace w2v {

constexpr int kGroupMaxLocal = 16;  // replicas one process drives (kernel argument arrays)

struct PtrList {
  float* p[kGroupMaxLocal];
};

// out = sum over n replicas' buffers, element-wise (float4).
__global__ void replica_sum_kernel(PtrList src, int n, float* out, int64_t n_elems) {
  const int64_t n4 = n_elems / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 acc = reinterpret_cast<const float4*>(src.p[0])[i];
    for (int k = 1; k < n; ++k) {
      const float4 v = reinterpret_cast<const float4*>(src.p[k])[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(out)[i] = acc;
  }
}

// out = sum over n replicas' arrays, element-wise (scalar: per-row counts at any offset).
__global__ void replica_sum1_kernel(PtrList src, int n, float* out, int64_t n_elems) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_elems; i += stride) {
    float acc = src.p[0][i];
    for (int k = 1; k < n; ++k) acc += src.p[k][i];
    out[i] = acc;
  }
}

// Per-row weight of the exchanged sum: 1 / max(1, contributors) (cnt) or s.
__device__ __forceinline__ float row_weight(const float* cnt, float s, int64_t i4, int64_t pitch) {
  return cnt ? 1.0f / fmaxf(1.0f, cnt[(i4 * 4) / pitch]) : s;
}

// Round boundary on one replica's matrix (element-wise, float4):
//   D_new = M - P                        (this round's own updates)
//   M     = M + w A - D_old  (fold)      (the pending exchange; fold == 0: none)
//   P     = M
__global__ void replica_delta_kernel(float* M, float* P, float* D, const float* A, const float* cnt, float s, int fold,
                                     int64_t pitch, int64_t n_elems) {
  const int64_t n4 = n_elems / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 m = reinterpret_cast<float4*>(M)[i];
    const float4 p = reinterpret_cast<const float4*>(P)[i];
    float4 dn = m;
    dn.x -= p.x; dn.y -= p.y; dn.z -= p.z; dn.w -= p.w;
    if (fold) {
      const float w = row_weight(cnt, s, i, pitch);
      const float4 a = reinterpret_cast<const float4*>(A)[i];
      const float4 d = reinterpret_cast<const float4*>(D)[i];
      m.x += w * a.x - d.x; m.y += w * a.y - d.y; m.z += w * a.z - d.z; m.w += w * a.w - d.w;
      reinterpret_cast<float4*>(M)[i] = m;
    }
    reinterpret_cast<float4*>(P)[i] = m;
    reinterpret_cast<float4*>(D)[i] = dn;
  }
}

// Fold the exchange into the replica on its own (the pending exchange covers
// other rows than the one being issued, or none is issued: finish): the same
// increment x = w A - D goes into M and into the snapshot P. M may already
// hold updates trained after the exchange was issued (overlap); P = M would
// absorb them and the next delta M - P would never carry them to the other
// replicas, while P += x keeps them in M - P.
__global__ void replica_fold_kernel(float* M, float* P, const float* D, const float* A, const float* cnt, float s,
                                    int64_t pitch, int64_t n_elems) {
  const int64_t n4 = n_elems / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float w = row_weight(cnt, s, i, pitch);
    float4 m = reinterpret_cast<float4*>(M)[i];
    float4 p = reinterpret_cast<float4*>(P)[i];
    const float4 a = reinterpret_cast<const float4*>(A)[i];
    const float4 d = reinterpret_cast<const float4*>(D)[i];
    const float4 x = make_float4(w * a.x - d.x, w * a.y - d.y, w * a.z - d.z, w * a.w - d.w);
    m.x += x.x; m.y += x.y; m.z += x.z; m.w += x.w;
    p.x += x.x; p.y += x.y; p.z += x.z; p.w += x.w;
    reinterpret_cast<float4*>(M)[i] = m;
    reinterpret_cast<float4*>(P)[i] = p;
  }
}

// F[r] = 1 if row r of D is not all zero (this replica changed the row), else 0.
__global__ void row_touch_kernel(const float* D, int64_t pitch, int64_t rows, float* F) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += stride) {
    const float4* q = reinterpret_cast<const float4*>(D + r * pitch);
    bool any = false;
    for (int64_t j = 0; j < pitch / 4 && !any; ++j) {
      const float4 v = q[j];
      any = v.x != 0.f || v.y != 0.f || v.z != 0.f || v.w != 0.f;
    }
    F[r] = any ? 1.0f : 0.0f;
  }
}

// One wavefront per row: sum of squares of the row's pitch floats (float4
// loads across the lanes, shuffle reduction).
__device__ __forceinline__ float row_sumsq(const float* row, int64_t pitch) {
  const int lane = (int)(threadIdx.x & 63);
  const float4* q = reinterpret_cast<const float4*>(row);
  float acc = 0.f;
  for (int64_t j = lane; j < pitch / 4; j += 64) {
    const float4 v = q[j];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  return acc;
}

// F[r] = |row r of D|^2 (this replica's update of the row this round).
__global__ void row_norm2_kernel(const float* D, int64_t pitch, int64_t rows, float* F) {
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; r < rows; r += waves) {
    const float ss = row_sumsq(D + r * pitch, pitch);
    if ((threadIdx.x & 63) == 0) F[r] = ss;
  }
}

// W2V_GROUP_ADAPTIVE: FA[r] (the sum over replicas of |D_i,r|^2) becomes the
// row's coherence c = |A_r|^2 / FA[r] in [0, R] (A = sum of the D_i): c = R
// when the replicas moved the row identically, 1 when their moves were
// orthogonal. The fold divides the row's summed update by max(1, c)
// (row_weight): the mean where the replicas agree, the sum where they are
// independent.
__global__ void row_coherence_kernel(const float* A, int64_t pitch, int64_t rows, float* FA) {
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; r < rows; r += waves) {
    const float ss = row_sumsq(A + r * pitch, pitch);
    if ((threadIdx.x & 63) == 0) {
      const float den = FA[r];
      FA[r] = den > 0.f ? ss / den : 1.0f;
    }
  }
}

}  // namespace w2v

namespace {

constexpr int kGrid = 2048, kBlock = 256;

struct Member {
  w2v_dev* h = nullptr;
  int device = 0;
  hipStream_t train = nullptr;   // the handle's stream (slices, deltas, folds)
  hipStream_t comm = nullptr;    // overlapped all-reduces
  hipEvent_t ready = nullptr;    // deltas extracted (train -> comm / replica 0)
  hipEvent_t done = nullptr;     // summed deltas ready (comm -> train)
  ncclComm_t nccl = nullptr;
  float* mat[3] = {nullptr, nullptr, nullptr};  // W, C, synapses1 (device, pitch-padded rows)
  float* P[3] = {nullptr, nullptr, nullptr};    // the shared model at the last exchange
  float* D[3] = {nullptr, nullptr, nullptr};    // this replica's updates of the round being exchanged
  float* A[3] = {nullptr, nullptr, nullptr};    // sum over replicas of D (same device: replica 0's only)
  float* F[3] = {nullptr, nullptr, nullptr};    // rows this replica changed (ROW_AVERAGE)
  float* FA[3] = {nullptr, nullptr, nullptr};   // contributors per row, summed (same device: replica 0's only)
  float* WC[3] = {nullptr, nullptr, nullptr};   // W2V_GROUP_SPLIT / SATURATION: per-row divisor in [1, nranks]
};

}  // namespace

struct w2v_group {
  std::vector<Member> m;
  int nranks = 1;
  bool local = false;       // every replica in this process, on one device: summing kernels, no RCCL
  bool exchange = false;    // rounds exchange anything: > 1 rank, or a communicator was asked for (unique id;
                            // one rank still runs the full RCCL round trip, which is how one GPU tests it)
  bool overlap = false;
  int32_t mode = W2V_GROUP_SUM;
  int64_t pitch = 0;
  bool pending = false;     // an overlapped exchange is in flight
  int64_t elems[3] = {0, 0, 0};  // floats per matrix (rows x pitch), 0 = unused
  int64_t rounds = 0;       // exchanges issued
  int64_t split_rows = 0;   // W2V_GROUP_SPLIT / SATURATION: rows (all matrices) with a divisor > 1
  float scale() const { return mode == W2V_GROUP_AVERAGE ? 1.0f / (float)nranks : 1.0f; }
  bool rows_counted() const { return mode == W2V_GROUP_ROW_AVERAGE || mode == W2V_GROUP_ADAPTIVE; }
  bool adaptive() const { return mode == W2V_GROUP_ADAPTIVE; }
  bool row_divisors() const { return mode == W2V_GROUP_SPLIT || mode == W2V_GROUP_SATURATION; }
  int64_t rows(int k) const { return pitch > 0 ? elems[k] / pitch : 0; }
  // Rows each exchange covers (w2v_group_average_rows_async): matrix k's rows
  // [lo[k], lo[k] + n[k]); `cur` for the exchange being issued, `pend` for the
  // one in flight (its deltas and sums live at the same offsets).
  struct Span {
    int64_t lo[3] = {0, 0, 0}, n[3] = {0, 0, 0};
    bool operator==(const Span& o) const {
      for (int k = 0; k < 3; ++k)
        if (lo[k] != o.lo[k] || n[k] != o.n[k]) return false;
      return true;
    }
  } cur, pend;
  int64_t at(const Span& sp, int k) const { return sp.lo[k] * pitch; }    // element offset
  int64_t len(const Span& sp, int k) const { return sp.n[k] * pitch; }   // elements
};

namespace {

int fail_g(int code, const std::string& msg) { return w2v::set_error(code, msg); }

#define HIP_G(expr)                                                                      \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) return fail_g(W2V_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define NCCL_G(expr)                                                                     \
  do {                                                                                   \
    ncclResult_t r_ = (expr);                                                            \
    if (r_ != ncclSuccess) return fail_g(W2V_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

void free_member(Member& x) {
  (void)hipSetDevice(x.device);
  if (x.comm) (void)hipStreamSynchronize(x.comm);
  if (x.train) (void)hipStreamSynchronize(x.train);
  for (int k = 0; k < 3; ++k) {
    for (float** b : {&x.P[k], &x.D[k], &x.A[k], &x.F[k], &x.FA[k], &x.WC[k]}) {
      if (*b) (void)hipFree(*b);
      *b = nullptr;
    }
  }
  if (x.nccl) (void)ncclCommDestroy(x.nccl);
  if (x.ready) (void)hipEventDestroy(x.ready);
  if (x.done) (void)hipEventDestroy(x.done);
  if (x.comm) (void)hipStreamDestroy(x.comm);
  x.nccl = nullptr;
  x.ready = x.done = nullptr;
  x.comm = nullptr;
}

// The summed deltas / per-row divisors of replica i's matrix k over span sp.
const float* sum_of(const w2v_group* g, size_t i, int k, const w2v_group::Span& sp) {
  return (g->local ? g->m[0].A[k] : g->m[i].A[k]) + g->at(sp, k);
}
const float* count_of(const w2v_group* g, size_t i, int k, const w2v_group::Span& sp) {
  if (g->row_divisors()) return g->m[i].WC[k] + sp.lo[k];
  if (!g->rows_counted()) return nullptr;
  return (g->local ? g->m[0].FA[k] : g->m[i].FA[k]) + sp.lo[k];
}

// Fold a finished exchange into every replica (train streams): M += s A - D, P = M.
int fold_pending(w2v_group* g) {
  if (!g->pending) return W2V_OK;
  for (size_t i = 0; i < g->m.size(); ++i) {
    Member& x = g->m[i];
    HIP_G(hipSetDevice(x.device));
    HIP_G(hipStreamWaitEvent(x.train, g->local ? g->m[0].done : x.done, 0));
    const w2v_group::Span& sp = g->pend;
    for (int k = 0; k < 3; ++k)
      if (sp.n[k]) {
        const int64_t o = g->at(sp, k);
        hipLaunchKernelGGL(w2v::replica_fold_kernel, dim3(kGrid), dim3(kBlock), 0, x.train, x.mat[k] + o, x.P[k] + o,
                           x.D[k] + o, sum_of(g, i, k, sp), count_of(g, i, k, sp), g->scale(), g->pitch, g->len(sp, k));
        HIP_G(hipGetLastError());
      }
  }
  g->pending = false;
  return W2V_OK;
}

// Sum the replicas' D into A: RCCL (one group over replicas and matrices) or,
// on one device, a kernel on replica 0's stream `s0`; `on_comm` selects the
// communication streams (overlap) or the training streams.
int sum_deltas(w2v_group* g, bool on_comm) {
  const size_t n = g->m.size();
  if (g->local) {
    Member& x0 = g->m[0];
    hipStream_t s0 = on_comm ? x0.comm : x0.train;
    HIP_G(hipSetDevice(x0.device));
    for (auto& x : g->m) HIP_G(hipStreamWaitEvent(s0, x.ready, 0));
    const w2v_group::Span& sp = g->cur;
    for (int k = 0; k < 3; ++k)
      if (sp.n[k]) {
        const int64_t o = g->at(sp, k), lo = sp.lo[k];
        w2v::PtrList pl{};
        for (size_t i = 0; i < n; ++i) pl.p[i] = g->m[i].D[k] + o;
        hipLaunchKernelGGL(w2v::replica_sum_kernel, dim3(kGrid), dim3(kBlock), 0, s0, pl, (int)n, x0.A[k] + o,
                           g->len(sp, k));
        HIP_G(hipGetLastError());
        if (g->rows_counted()) {
          for (size_t i = 0; i < n; ++i) pl.p[i] = g->m[i].F[k] + lo;
          hipLaunchKernelGGL(w2v::replica_sum1_kernel, dim3(kGrid), dim3(kBlock), 0, s0, pl, (int)n, x0.FA[k] + lo,
                             sp.n[k]);
          HIP_G(hipGetLastError());
        }
        if (g->adaptive()) {
          hipLaunchKernelGGL(w2v::row_coherence_kernel, dim3(kGrid), dim3(kBlock), 0, s0, x0.A[k] + o, g->pitch,
                             sp.n[k], x0.FA[k] + lo);
          HIP_G(hipGetLastError());
        }
      }
    HIP_G(hipEventRecord(x0.done, s0));
    return W2V_OK;
  }
  for (auto& x : g->m)
    if (on_comm) {
      HIP_G(hipSetDevice(x.device));
      HIP_G(hipStreamWaitEvent(x.comm, x.ready, 0));
    }
  const w2v_group::Span& sp = g->cur;
  NCCL_G(ncclGroupStart());
  for (auto& x : g->m) {
    (void)hipSetDevice(x.device);
    for (int k = 0; k < 3; ++k)
      if (sp.n[k]) {
        const int64_t o = g->at(sp, k), lo = sp.lo[k];
        ncclResult_t r = ncclAllReduce(x.D[k] + o, x.A[k] + o, (size_t)g->len(sp, k), ncclFloat32, ncclSum, x.nccl,
                                       on_comm ? x.comm : x.train);
        if (r == ncclSuccess && g->rows_counted())
          r = ncclAllReduce(x.F[k] + lo, x.FA[k] + lo, (size_t)sp.n[k], ncclFloat32, ncclSum, x.nccl,
                            on_comm ? x.comm : x.train);
        if (r != ncclSuccess) {
          (void)ncclGroupEnd();
          return fail_g(W2V_ERR_COMM, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        }
      }
  }
  NCCL_G(ncclGroupEnd());
  for (auto& x : g->m) {
    HIP_G(hipSetDevice(x.device));
    hipStream_t st = on_comm ? x.comm : x.train;
    if (g->adaptive())
      for (int k = 0; k < 3; ++k)
        if (sp.n[k]) {
          hipLaunchKernelGGL(w2v::row_coherence_kernel, dim3(kGrid), dim3(kBlock), 0, st, x.A[k] + g->at(sp, k),
                             g->pitch, sp.n[k], x.FA[k] + sp.lo[k]);
          HIP_G(hipGetLastError());
        }
    HIP_G(hipEventRecord(x.done, st));
  }
  return W2V_OK;
}

// One exchange over g->cur (set by the callers below).
int exchange(w2v_group* g) {
  if (!g->exchange) return W2V_OK;
  ++g->rounds;
  // extract this round's deltas and fold the pending exchange in (overlap):
  // fused into the delta kernel when the pending exchange covers the same
  // rows, else folded first on its own rows
  if (g->overlap && g->pending && !(g->pend == g->cur))
    if (int rc = fold_pending(g)) return rc;
  const bool fold = g->overlap && g->pending;
  if (fold)
    for (size_t i = 0; i < g->m.size(); ++i) {
      Member& x = g->m[i];
      HIP_G(hipSetDevice(x.device));
      HIP_G(hipStreamWaitEvent(x.train, g->local ? g->m[0].done : x.done, 0));
    }
  const w2v_group::Span& sp = g->cur;
  for (size_t i = 0; i < g->m.size(); ++i) {
    Member& x = g->m[i];
    HIP_G(hipSetDevice(x.device));
    for (int k = 0; k < 3; ++k)
      if (sp.n[k]) {
        const int64_t o = g->at(sp, k), lo = sp.lo[k];
        hipLaunchKernelGGL(w2v::replica_delta_kernel, dim3(kGrid), dim3(kBlock), 0, x.train, x.mat[k] + o, x.P[k] + o,
                           x.D[k] + o, fold ? sum_of(g, i, k, sp) : nullptr, fold ? count_of(g, i, k, sp) : nullptr,
                           g->scale(), fold ? 1 : 0, g->pitch, g->len(sp, k));
        HIP_G(hipGetLastError());
        if (g->adaptive()) {
          hipLaunchKernelGGL(w2v::row_norm2_kernel, dim3(kGrid), dim3(kBlock), 0, x.train, x.D[k] + o, g->pitch,
                             sp.n[k], x.F[k] + lo);
          HIP_G(hipGetLastError());
        } else if (g->rows_counted()) {
          hipLaunchKernelGGL(w2v::row_touch_kernel, dim3(kGrid), dim3(kBlock), 0, x.train, x.D[k] + o, g->pitch,
                             sp.n[k], x.F[k] + lo);
          HIP_G(hipGetLastError());
        }
      }
    HIP_G(hipEventRecord(x.ready, x.train));
  }
  g->pending = false;
  if (int rc = sum_deltas(g, g->overlap)) return rc;
  g->pending = true;
  g->pend = g->cur;
  if (!g->overlap) return fold_pending(g);  // blocking: fold in right away, on the training streams
  return W2V_OK;
}

}  // namespace

extern "C" {

int w2v_group_unique_id(uint8_t* id) {
  if (!id) return fail_g(W2V_ERR_ARG, "w2v_group_unique_id: null argument");
  static_assert(sizeof(ncclUniqueId) == W2V_GROUP_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  NCCL_G(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return W2V_OK;
}

int w2v_group_create(w2v_dev** members, int32_t n, const uint8_t* unique_id, int32_t nranks, int32_t first_rank,
                     w2v_group** out) {
  w2v::Range range_("w2v_group_create");
  if (!members || !out || n < 1) return fail_g(W2V_ERR_ARG, "w2v_group_create: need >= 1 member handle");
  *out = nullptr;
  if (n > w2v::kGroupMaxLocal) return fail_g(W2V_ERR_UNSUPPORTED, "w2v_group_create: at most 16 replicas per process");
  if (!unique_id) {
    nranks = n;
    first_rank = 0;
  }
  if (nranks < n || first_rank < 0 || first_rank + n > nranks)
    return fail_g(W2V_ERR_ARG, "w2v_group_create: ranks [first_rank, first_rank + n) must lie in [0, nranks)");
  w2v_group* g = new w2v_group();
  g->nranks = nranks;
  for (int i = 0; i < n; ++i) {
    w2v_dev* h = members[i];
    Member x;
    x.h = h;
    int64_t pitch = 0;
    if (!h || w2v_dev_model_layout(h, &x.mat[0], &x.mat[1], &x.mat[2], &pitch) != W2V_OK) {
      w2v_group_destroy(g);
      return fail_g(W2V_ERR_STATE, "w2v_group_create: every member needs its vocab and model resident");
    }
    w2v::DevInfo info = w2v::dev_info(h);
    x.device = info.device;
    x.train = info.stream;
    g->pitch = pitch;
    const int64_t e[3] = {info.V * pitch, x.mat[1] ? info.V * pitch : 0,
                          x.mat[2] ? std::max<int64_t>(info.V - 1, 0) * pitch : 0};
    for (int k = 0; k < 3; ++k) {
      if (i == 0) g->elems[k] = e[k];
      else if (g->elems[k] != e[k]) {
        w2v_group_destroy(g);
        return fail_g(W2V_ERR_ARG, "w2v_group_create: members must hold models of the same shape");
      }
    }
    g->m.push_back(x);
  }
  bool same = true;
  for (auto& x : g->m) same = same && x.device == g->m[0].device;
  g->local = n > 1 && same && !unique_id;
  g->exchange = nranks > 1 || unique_id != nullptr;
  for (size_t i = 0; i < g->m.size(); ++i) {
    Member& x = g->m[i];
    bool ok = hipSetDevice(x.device) == hipSuccess &&
              hipStreamCreateWithFlags(&x.comm, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&x.ready, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&x.done, hipEventDisableTiming) == hipSuccess;
    // P (the shared model: every replica starts from the same weights), D, A
    for (int k = 0; k < 3 && ok && g->exchange; ++k) {
      if (!g->elems[k]) continue;
      const size_t bytes = (size_t)g->elems[k] * sizeof(float);
      const size_t fbytes = (size_t)((g->elems[k] / g->pitch + 3) & ~int64_t(3)) * sizeof(float);  // rows, float4-padded
      const bool own_sum = !(g->local && i > 0);
      ok = hipMalloc(&x.P[k], bytes) == hipSuccess && hipMalloc(&x.D[k], bytes) == hipSuccess &&
           (!own_sum || hipMalloc(&x.A[k], bytes) == hipSuccess) && hipMalloc(&x.F[k], fbytes) == hipSuccess &&
           hipMemsetAsync(x.F[k], 0, fbytes, x.train) == hipSuccess &&
           (!own_sum || hipMalloc(&x.FA[k], fbytes) == hipSuccess) &&
           hipMemcpyAsync(x.P[k], x.mat[k], bytes, hipMemcpyDeviceToDevice, x.train) == hipSuccess;
    }
    if (!ok) {
      w2v_group_destroy(g);
      return fail_g(W2V_ERR_HIP, "w2v_group_create: stream / event / exchange buffer setup failed (out of memory?)");
    }
  }
  if (!g->local && g->exchange) {
    ncclResult_t r = ncclSuccess;
    if (!unique_id) {
      std::vector<int> devs;
      for (auto& x : g->m) devs.push_back(x.device);
      std::vector<ncclComm_t> comms(devs.size());
      r = ncclCommInitAll(comms.data(), (int)devs.size(), devs.data());
      if (r == ncclSuccess)
        for (size_t i = 0; i < comms.size(); ++i) g->m[i].nccl = comms[i];
    } else {
      ncclUniqueId u;
      std::memcpy(&u, unique_id, sizeof(u));
      r = ncclGroupStart();
      for (int i = 0; i < n && r == ncclSuccess; ++i) {
        (void)hipSetDevice(g->m[i].device);
        r = ncclCommInitRank(&g->m[i].nccl, nranks, u, first_rank + i);
      }
      const ncclResult_t r2 = ncclGroupEnd();
      if (r == ncclSuccess) r = r2;
    }
    if (r != ncclSuccess) {
      w2v_group_destroy(g);
      return fail_g(W2V_ERR_COMM, std::string("w2v_group_create: RCCL communicator: ") + ncclGetErrorString(r));
    }
  }
  for (auto& x : g->m)  // the shared-model copies P are taken before the caller touches the replicas again
    if (hipSetDevice(x.device) != hipSuccess || hipStreamSynchronize(x.train) != hipSuccess) {
      w2v_group_destroy(g);
      return fail_g(W2V_ERR_HIP, "w2v_group_create: synchronising the replicas failed");
    }
  for (auto& x : g->m) w2v::set_replicas(x.h, nranks);
  *out = g;
  return W2V_OK;
}

void w2v_group_destroy(w2v_group* g) {
  if (!g) return;
  for (auto& x : g->m) free_member(x);
  delete g;
}

int w2v_group_set_overlap(w2v_group* g, int32_t on) {
  if (!g) return fail_g(W2V_ERR_ARG, "null group");
  if (g->pending) return fail_g(W2V_ERR_STATE, "w2v_group_set_overlap: an exchange is in flight (w2v_group_finish first)");
  g->overlap = on != 0;
  return W2V_OK;
}

int w2v_group_set_mode(w2v_group* g, int32_t mode) {
  if (!g) return fail_g(W2V_ERR_ARG, "null group");
  if (mode != W2V_GROUP_SUM && mode != W2V_GROUP_AVERAGE && mode != W2V_GROUP_ROW_AVERAGE &&
      mode != W2V_GROUP_ADAPTIVE)
    return fail_g(W2V_ERR_ARG, "bad group mode (W2V_GROUP_SPLIT is set by w2v_group_set_split)");
  if (g->pending) return fail_g(W2V_ERR_STATE, "w2v_group_set_mode: an exchange is in flight (w2v_group_finish first)");
  g->mode = mode;
  return W2V_OK;
}

}  // extern "C"

namespace {
// Per-row divisors of the summed update from member 0's corpus statistics
// (every replica trains the same vocabulary on a shard of the same corpus):
// c = divisor(u), u = the row's expected updates per replica in a round of
// tokens_per_round raw tokens.
template <class F>
int set_row_divisors(w2v_group* g, int64_t tokens_per_round, int32_t mode, F divisor, const char* what) {
  if (g->pending) return fail_g(W2V_ERR_STATE, std::string(what) + ": an exchange is in flight (w2v_group_finish first)");
  std::vector<float> wc[3];
  for (int k = 0; k < 3; ++k) {
    if (!g->elems[k]) continue;
    std::vector<double> rate;
    if (!w2v::row_update_rates(g->m[0].h, k, rate) || (int64_t)rate.size() != g->rows(k))
      return fail_g(W2V_ERR_STATE, std::string(what) + ": the replicas need their vocab and corpus statistics uploaded");
    wc[k].resize(rate.size());
    for (size_t r = 0; r < rate.size(); ++r) wc[k][r] = divisor(rate[r] * (double)tokens_per_round);
  }
  for (auto& x : g->m) {
    HIP_G(hipSetDevice(x.device));
    for (int k = 0; k < 3; ++k) {
      if (!g->elems[k]) continue;
      if (!x.WC[k]) HIP_G(hipMalloc(&x.WC[k], wc[k].size() * sizeof(float)));
      HIP_G(hipMemcpy(x.WC[k], wc[k].data(), wc[k].size() * sizeof(float), hipMemcpyHostToDevice));
    }
  }
  int64_t avg = 0;
  for (int k = 0; k < 3; ++k)
    for (float w : wc[k]) avg += w > 1.0f;
  g->split_rows = avg;
  g->mode = mode;
  return W2V_OK;
}
}  // namespace

extern "C" {

int w2v_group_set_split(w2v_group* g, int64_t tokens_per_round, float saturated_updates) {
  w2v::Range range_("w2v_group_set_split");
  if (!g) return fail_g(W2V_ERR_ARG, "null group");
  if (tokens_per_round < 1 || !(saturated_updates >= 0.0f))
    return fail_g(W2V_ERR_ARG, "w2v_group_set_split: tokens_per_round >= 1 and saturated_updates >= 0");
  const float R = (float)g->nranks;
  return set_row_divisors(g, tokens_per_round, W2V_GROUP_SPLIT,
                          [&](double u) { return u >= (double)saturated_updates ? R : 1.0f; }, "w2v_group_set_split");
}

// W2V_GROUP_SATURATION. A row that one model would update n times in a round,
// each update contracting its distance to the row's current optimum by a
// factor (1 - beta), moves 1 - (1 - beta)^n of the way; R replicas that each
// update it u = n / R times from the same start move R (1 - (1 - beta)^u) in
// sum. The divisor c = R (1 - (1 - beta)^u) / (1 - (1 - beta)^(R u)) makes the
// exchanged move the one model's: c -> 1 (the sum) for rows in the linear
// regime (u beta << 1: independent small updates add), c -> R (the mean) for
// rows every replica drives to the same optimum within the round (summing R
// such moves overshoots R-fold, which is GD past its stability bound for R > 2).
int w2v_group_set_saturation(w2v_group* g, int64_t tokens_per_round, float beta) {
  w2v::Range range_("w2v_group_set_saturation");
  if (!g) return fail_g(W2V_ERR_ARG, "null group");
  if (tokens_per_round < 1 || !(beta > 0.0f && beta < 1.0f))
    return fail_g(W2V_ERR_ARG, "w2v_group_set_saturation: tokens_per_round >= 1 and 0 < beta < 1");
  const double R = (double)g->nranks, lb = std::log1p(-(double)beta);
  return set_row_divisors(g, tokens_per_round, W2V_GROUP_SATURATION, [&](double u) {
    const double a = -std::expm1(u * lb), b = -std::expm1(R * u * lb);
    const double c = b > 0.0 ? R * a / b : 1.0;
    return (float)std::min(R, std::max(1.0, c));
  }, "w2v_group_set_saturation");
}

int w2v_group_average_async(w2v_group* g) {
  w2v::Range range_("w2v_group_average_async");
  if (!g) return fail_g(W2V_ERR_ARG, "null group");
  for (int k = 0; k < 3; ++k) {
    g->cur.lo[k] = 0;
    g->cur.n[k] = g->rows(k);
  }
  return exchange(g);
}

int w2v_group_average_rows_async(w2v_group* g, int64_t rows) {
  w2v::Range range_("w2v_group_average_rows_async");
  if (!g) return fail_g(W2V_ERR_ARG, "null group");
  if (rows < 0) return fail_g(W2V_ERR_ARG, "w2v_group_average_rows_async: rows must be >= 0");
  for (int k = 0; k < 3; ++k) {  // W / C: the first rows (the most frequent words); synapses1: the nodes nearest the root
    const int64_t R = g->rows(k), n = rows == 0 ? R : std::min(rows, R);
    g->cur.lo[k] = k == 2 ? R - n : 0;
    g->cur.n[k] = n;
  }
  return exchange(g);
}

int w2v_group_finish(w2v_group* g) {
  w2v::Range range_("w2v_group_finish");
  if (!g) return fail_g(W2V_ERR_ARG, "null group");
  if (int rc = fold_pending(g)) return rc;
  for (auto& x : g->m) {
    HIP_G(hipSetDevice(x.device));
    HIP_G(hipStreamSynchronize(x.train));
    HIP_G(hipStreamSynchronize(x.comm));
  }
  return W2V_OK;
}

int w2v_group_row_divisors(w2v_group* g, int32_t which, float* out, int64_t n) {
  if (!g || !out) return fail_g(W2V_ERR_ARG, "null argument");
  if (which < 0 || which > 2 || !g->elems[which]) return fail_g(W2V_ERR_ARG, "no such matrix in the group");
  if (n != g->rows(which)) return fail_g(W2V_ERR_ARG, "n must be the matrix's row count");
  if (!g->row_divisors()) {
    std::fill(out, out + n, 1.0f);
    return W2V_OK;
  }
  HIP_G(hipSetDevice(g->m[0].device));
  HIP_G(hipMemcpy(out, g->m[0].WC[which], (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
  return W2V_OK;
}

int w2v_group_split_rows(w2v_group* g, int64_t* rows) {
  if (!g || !rows) return fail_g(W2V_ERR_ARG, "null argument");
  *rows = g->row_divisors() ? g->split_rows : 0;
  return W2V_OK;
}

int w2v_group_info(w2v_group* g, int32_t* nranks, int32_t* local, int32_t* overlap, int64_t* rounds) {
  if (!g) return fail_g(W2V_ERR_ARG, "null group");
  if (nranks) *nranks = g->nranks;
  if (local) *local = g->local ? 1 : 0;
  if (overlap) *overlap = g->overlap ? 1 : 0;
  if (rounds) *rounds = g->rounds;
  return W2V_OK;
}

}  // extern "C"
