// w2v_ingest.hip — corpus ingestion on the GPU (include/w2v_ingest.h): the
// vocabulary count (Word2Vec.cpp:134-141) and build_sample's id mapping
// (:212-230) of a corpus file, bit-exact with the host readers
// (csrc/host/corpus.cpp, which match line_docs, Word2Vec.cpp:19-30, and the
// CLI's text8 reader, main.cpp:63-92).
//
// Per chunk of the file (cut after a whitespace byte, after '\n' for lines):
//   * token starts: a byte that is not C-locale whitespace after one that is
//     (or at the chunk start) — flags, then a device select into positions;
//   * per token (one thread): its end, two 64-bit hashes of its bytes, and the
//     newlines between it and the next token (the line index of a token is
//     the newlines before it: a scan of those counts);
//   * pass 1, insert: find or claim the token's slot in an open-addressing
//     table keyed by the first hash (compare-and-swap on the key) and lower
//     the slot's first byte offset (atomic min, only when smaller: after the
//     first occurrences nearly every token only reads). Idempotent, so a
//     chunk that fills the table past half is re-inserted after the table
//     doubles (rehash kernel);
//   * pass 1, count: one add per token on its slot, aggregated per workgroup
//     in an LDS table first (Zipf corpora: the hot words' adds stay in LDS,
//     one global add per distinct word per workgroup);
//   * the used slots, sorted by first occurrence on the device (select +
//     radix sort), are the words in the order the host map needs;
//   * pass 2: look the token up, check the second hash and the length against
//     the slot's (a collision of the first hash between two different words
//     fails the call rather than merging them), map to the vocab index, and
//     append the in-vocab ids (a device select). Sentence offsets without
//     atomics: the exclusive scan of the kept flags gives each token's output
//     position, and the token that opens sentence s writes offsets[s] (text8:
//     raw token index 1000 s; lines: the first token of a line, which also
//     writes the offsets of the empty lines before it).
// The per-word token histogram the training handle needs (flush scales,
// w2v_dev_adopt_corpus) is the vocab words' counts from pass 1.
// The work is byte- and hash-table-bound, far from the HBM roofline: the
// point is taking the counting and mapping of a multi-GB corpus off the host.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "w2v_dev_internal.hpp"
#include "w2v_ingest.h"

namespace w2v {
namespace ingest {

constexpr uint64_t kEmpty = 0;
constexpr int64_t kText8Sentence = 1000;  // main.cpp:66
constexpr int kMaxProbe = 4096;           // a longer chain counts as a full table (the table grows)
constexpr int kBlock = 256;
constexpr int kLdsSlots = 4096;  // per-workgroup count aggregation
constexpr uint32_t kLdsEmpty = 0xFFFFFFFFu;
constexpr int64_t kResidentMax = (int64_t)64 << 30;  // default: bytes of corpus kept in HBM between the passes

__device__ __forceinline__ bool is_space(unsigned char c) {  // C-locale isspace, as operator>>
  return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

// Token starts, compacted without a byte-flag array: a workgroup takes a
// 4 KiB tile (16 bytes per thread), counts its starts (pass a), the tile
// counts are scanned, and the workgroup writes its starts in order (pass b).
constexpr int kTileBytes = 4096;
constexpr int kPerThread = kTileBytes / 256;

__device__ __forceinline__ int starts_in(const unsigned char* b, int64_t n, int64_t i0, uint32_t* mask) {
  int c = 0;
  uint32_t m = 0;
  *mask = 0;
  if (i0 >= n) return 0;
  bool prev_space = i0 == 0 ? true : is_space(b[i0 - 1]);
  for (int k = 0; k < kPerThread; ++k) {
    const int64_t i = i0 + k;
    if (i >= n) break;
    const bool sp = is_space(b[i]);
    if (!sp && prev_space) {
      ++c;
      m |= 1u << k;
    }
    prev_space = sp;
  }
  *mask = m;
  return c;
}

__global__ __launch_bounds__(256) void tile_count_kernel(const unsigned char* b, int64_t n, int64_t* tile_count) {
  __shared__ int sum;
  if (threadIdx.x == 0) sum = 0;
  __syncthreads();
  uint32_t m;
  const int c = starts_in(b, n, (int64_t)blockIdx.x * kTileBytes + (int64_t)threadIdx.x * kPerThread, &m);
  if (c) atomicAdd(&sum, c);
  __syncthreads();
  if (threadIdx.x == 0) tile_count[blockIdx.x] = sum;
}

__global__ __launch_bounds__(256) void tile_write_kernel(const unsigned char* b, int64_t n, const int64_t* tile_pos,
                                                         int64_t* starts) {
  __shared__ int sh[256];
  uint32_t m;
  const int64_t i0 = (int64_t)blockIdx.x * kTileBytes + (int64_t)threadIdx.x * kPerThread;
  const int c = starts_in(b, n, i0, &m);
  sh[threadIdx.x] = c;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {  // inclusive scan of the per-thread counts
    const int v = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : 0;
    __syncthreads();
    sh[threadIdx.x] += v;
    __syncthreads();
  }
  int64_t pos = tile_pos[blockIdx.x] + sh[threadIdx.x] - c;
  while (m) {
    const int k = __builtin_ctz(m);
    m &= m - 1;
    starts[pos++] = i0 + k;
  }
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// One token: its length, two hashes, and the newlines before the next token.
struct Tok {
  uint32_t len;
  uint32_t nl_after;
  uint64_t h1, h2;
};

__device__ __forceinline__ Tok read_token(const unsigned char* b, int64_t n, int64_t s) {
  Tok t;
  uint64_t f = 1469598103934665603ull;  // FNV-1a
  uint64_t m = 0x9E3779B97F4A7C15ull;   // multiplicative rolling hash, another prime
  int64_t e = s;
  while (e < n && !is_space(b[e])) {
    const unsigned char c = b[e];
    f = (f ^ c) * 1099511628211ull;
    m = (m + c + 1) * 0xC2B2AE3D27D4EB4Full;
    ++e;
  }
  t.len = (uint32_t)(e - s);
  t.h1 = mix64(f ^ (uint64_t)t.len);
  if (t.h1 == kEmpty) t.h1 = 1;
  t.h2 = mix64(m + 0x165667B19E3779F9ull * (uint64_t)t.len);
  uint32_t nl = 0;
  while (e < n && is_space(b[e])) {
    nl += b[e] == '\n';
    ++e;
  }
  t.nl_after = nl;
  return t;
}

struct Table {
  uint64_t* key;  // first hash, 0 = empty
  uint64_t* h2;
  unsigned long long* first;  // smallest byte offset seen
  unsigned long long* count;
  uint32_t* len;
  uint64_t mask;
};

// Claim (CAS) or find key h1 from its home slot; -1 after kMaxProbe slots.
__device__ __forceinline__ int64_t claim(const Table& tab, uint64_t h1, bool* won) {
  uint64_t i = h1 & tab.mask;
  *won = false;
  for (int probe = 0; probe < kMaxProbe; ++probe, i = (i + 1) & tab.mask) {
    uint64_t cur = __hip_atomic_load(&tab.key[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == kEmpty) {
      uint64_t expected = kEmpty;
      if (__hip_atomic_compare_exchange_strong(&tab.key[i], &expected, h1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        *won = true;
        return (int64_t)i;
      }
      cur = expected;
    }
    if (cur == h1) return (int64_t)i;
  }
  return -1;
}

// Pass 1, insert (idempotent). base_off: the chunk's byte offset in the file.
__global__ void insert_kernel(const unsigned char* b, int64_t n, const int64_t* starts, int64_t nt, int64_t base_off,
                              Table tab, uint32_t* slot, uint32_t* nl_after, unsigned long long* used,
                              unsigned long long* fail) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += stride) {
    const int64_t s = starts[t];
    const Tok k = read_token(b, n, s);
    nl_after[t] = k.nl_after;
    bool won = false;
    const int64_t i = claim(tab, k.h1, &won);
    if (i < 0) {
      atomicAdd(fail, 1ull);
      continue;
    }
    if (won) {
      tab.h2[i] = k.h2;
      tab.len[i] = k.len;
      atomicAdd(used, 1ull);
    }
    const unsigned long long off = (unsigned long long)(base_off + s);
    if (off < __hip_atomic_load(&tab.first[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&tab.first[i], off);
    slot[t] = (uint32_t)i;
  }
}

// Move every used slot of `from` into `to` (a larger, empty table).
__global__ void rehash_kernel(Table from, int64_t from_cap, Table to, unsigned long long* fail) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < from_cap; i += stride) {
    const uint64_t h1 = from.key[i];
    if (h1 == kEmpty) continue;
    bool won = false;
    const int64_t j = claim(to, h1, &won);
    if (j < 0 || !won) {
      atomicAdd(fail, 1ull);
      continue;
    }
    to.h2[j] = from.h2[i];
    to.len[j] = from.len[i];
    to.first[j] = from.first[i];
    to.count[j] = from.count[i];
  }
}

// Pass 1, count: per workgroup, adds go to an LDS table of slots first; a
// slot that finds no LDS entry within 8 probes adds to HBM directly.
__global__ __launch_bounds__(kBlock) void count_kernel(const uint32_t* slot, int64_t nt, unsigned long long* count) {
  __shared__ uint32_t lkey[kLdsSlots];
  __shared__ uint32_t lcnt[kLdsSlots];
  for (int h = threadIdx.x; h < kLdsSlots; h += kBlock) {
    lkey[h] = kLdsEmpty;
    lcnt[h] = 0;
  }
  __syncthreads();
  const int64_t per = (nt + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = min(nt, lo + per);
  for (int64_t t = lo + threadIdx.x; t < hi; t += kBlock) {
    const uint32_t s = slot[t];
    uint32_t h = (s * 2654435761u) >> 20;  // 12 bits
    bool done = false;
    for (int probe = 0; probe < 8 && !done; ++probe, h = (h + 1) & (kLdsSlots - 1)) {
      uint32_t k = lkey[h];
      if (k == kLdsEmpty) {
        const uint32_t old = atomicCAS(&lkey[h], kLdsEmpty, s);
        k = old == kLdsEmpty ? s : old;  // claimed it, or another thread did
      }
      if (k == s) {
        atomicAdd(&lcnt[h], 1u);
        done = true;
      }
    }
    if (!done) atomicAdd(&count[s], 1ull);
  }
  __syncthreads();
  for (int h = threadIdx.x; h < kLdsSlots; h += kBlock)
    if (lcnt[h]) atomicAdd(&count[lkey[h]], (unsigned long long)lcnt[h]);
}

struct UsedSlot {
  const uint64_t* key;
  __host__ __device__ bool operator()(const int64_t& i) const { return key[i] != kEmpty; }
};

__global__ void gather_first_kernel(const int64_t* slots, int64_t m, const unsigned long long* first,
                                    unsigned long long* out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) out[k] = first[slots[k]];
}

__global__ void gather_words_kernel(const int64_t* order, int64_t m, Table tab, int64_t* first, int32_t* len,
                                    int64_t* count) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) {
    const int64_t s = order[k];
    first[k] = (int64_t)tab.first[s];
    len[k] = (int32_t)tab.len[s];
    count[k] = (int64_t)tab.count[s];
  }
}

__global__ void scatter_ids_kernel(const int64_t* order, const int32_t* vidx, int64_t m, int32_t* slot_id) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) slot_id[order[k]] = vidx[k];
}

// Pass 2: token -> vocab index (or -1) and its kept flag. Verifies the second hash and length.
__global__ void map_kernel(const unsigned char* b, int64_t n, const int64_t* starts, int64_t nt, Table tab,
                           const int32_t* slot_id, int32_t* tok_id, int32_t* kept, uint32_t* nl_after,
                           unsigned long long* mismatch) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += stride) {
    const Tok k = read_token(b, n, starts[t]);
    nl_after[t] = k.nl_after;
    uint64_t i = k.h1 & tab.mask;
    int32_t id = -1;
    bool found = false;
    for (uint64_t probe = 0; probe <= tab.mask; ++probe, i = (i + 1) & tab.mask) {
      const uint64_t cur = tab.key[i];
      if (cur == kEmpty) break;
      if (cur == k.h1) {
        found = true;
        if (tab.h2[i] != k.h2 || tab.len[i] != k.len) atomicAdd(mismatch, 1ull);
        id = slot_id[i];
        break;
      }
    }
    if (!found) atomicAdd(mismatch, 1ull);  // pass 2 saw a word pass 1 did not (different bytes)
    tok_id[t] = id;
    kept[t] = id >= 0 ? 1 : 0;
  }
}

// offsets[s] = kept tokens before sentence s, written by the token that opens s.
// text8: raw token 1000 s. lines: the first token of line L writes offsets[l]
// for l in (previous token's line, L] (the empty lines before it too).
__global__ void boundary_kernel(const int32_t* kpos, const int64_t* line_of, int64_t nt, int64_t raw_base,
                                int64_t kept_base, int64_t prev_line, int text8, int64_t* offsets) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += stride) {
    const int64_t pos = kept_base + kpos[t];
    if (text8) {
      const int64_t r = raw_base + t;
      if (r > 0 && r % kText8Sentence == 0) offsets[r / kText8Sentence] = pos;
    } else {
      const int64_t L = line_of[t];
      const int64_t P = t > 0 ? line_of[t - 1] : prev_line;
      for (int64_t l = P + 1; l <= L; ++l) offsets[l] = pos;
    }
  }
}

__global__ void fill_kernel(int64_t* p, int64_t lo, int64_t hi, int64_t v) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += stride) p[i] = v;
}

__global__ void add_base_kernel(int64_t* l, int64_t m, int64_t base) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < m; t += stride) l[t] += base;
}

struct NotNegative {
  __host__ __device__ bool operator()(const int32_t& v) const { return v >= 0; }
};

inline dim3 grid_for(int64_t n) {
  return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(8192, (n + kBlock - 1) / kBlock)));
}

}  // namespace ingest
}  // namespace w2v

using namespace w2v::ingest;

struct w2v_ingest {
  int device = 0;
  int format = W2V_INGEST_LINES;
  int64_t chunk = (int64_t)1 << 30;
  int64_t resident_max = kResidentMax;
  hipStream_t stream = nullptr;
  // hash table
  int64_t cap = 0;
  Table tab{};
  unsigned long long* ctr = nullptr;  // [0] used slots, [1] probe failures, [2] mismatches
  // pass 1 results
  bool counted = false;
  int64_t n_bytes = 0, raw_tokens = 0, n_sentences = 0, n_words = 0;
  int64_t* order = nullptr;  // device: the used slots in order of first occurrence
  std::vector<int64_t> word_count;  // host: pass-1 counts in that order
  // pass 2 results
  bool mapped = false;
  int32_t* ids = nullptr;
  int64_t n_ids = 0;
  int64_t* offsets = nullptr;  // n_sentences + 1
  std::vector<int64_t> hist;   // host: tokens per vocab id
  // chunk work buffers
  unsigned char* buf = nullptr;   // one chunk (the file is not resident)
  unsigned char* file = nullptr;  // the whole file in HBM between pass 1 and pass 2 (<= kResidentMax)
  int64_t file_n = -1;
  const unsigned char* cur = nullptr;  // device bytes of the current chunk
  int64_t* tile = nullptr;             // per-4 KiB-tile start counts, then positions
  int64_t* starts = nullptr;
  uint32_t* nl_after = nullptr;
  uint32_t* slot = nullptr;
  int64_t* line_of = nullptr;
  int32_t* tok_id = nullptr;
  int32_t* kept = nullptr;
  int32_t* kpos = nullptr;
  int64_t* n_sel = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  int64_t work_cap = 0;  // bytes the work buffers hold
};

namespace {

int fail_i(int code, const std::string& m) { return w2v::set_error(code, m); }

#define HIP_I(expr)                                                                                       \
  do {                                                                                                    \
    hipError_t e_ = (expr);                                                                               \
    if (e_ != hipSuccess) return fail_i(W2V_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

bool host_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }

// Chunks cut after a '\n' (lines) or a whitespace byte (text8), as corpus.cpp's split().
std::vector<std::pair<int64_t, int64_t>> chunks(const char* p, int64_t n, int64_t size, bool lines) {
  std::vector<std::pair<int64_t, int64_t>> r;
  int64_t b = 0;
  while (b < n) {
    int64_t e = std::min(n, b + size);
    while (e < n && !(lines ? p[e - 1] == '\n' : host_space(p[e - 1]))) ++e;
    r.emplace_back(b, e);
    b = e;
  }
  return r;
}

void free_table(Table& t) {
  dfree(t.key); dfree(t.h2); dfree(t.first); dfree(t.count); dfree(t.len);
}

int alloc_table(Table& t, int64_t cap, hipStream_t s) {
  HIP_I(hipMalloc(&t.key, cap * sizeof(uint64_t)));
  HIP_I(hipMalloc(&t.h2, cap * sizeof(uint64_t)));
  HIP_I(hipMalloc(&t.first, cap * sizeof(unsigned long long)));
  HIP_I(hipMalloc(&t.count, cap * sizeof(unsigned long long)));
  HIP_I(hipMalloc(&t.len, cap * sizeof(uint32_t)));
  HIP_I(hipMemsetAsync(t.key, 0, cap * sizeof(uint64_t), s));
  HIP_I(hipMemsetAsync(t.first, 0xFF, cap * sizeof(unsigned long long), s));
  HIP_I(hipMemsetAsync(t.count, 0, cap * sizeof(unsigned long long), s));
  t.mask = (uint64_t)cap - 1;
  return W2V_OK;
}

constexpr int64_t kMaxCap = (int64_t)1 << 30;

// Double the table until it holds `need` words at most half full.
int grow(w2v_ingest* g, int64_t need) {
  int64_t cap = g->cap * 2;
  while (cap < 2 * need) cap <<= 1;
  if (cap > kMaxCap) return fail_i(W2V_ERR_UNSUPPORTED, "w2v_ingest_count: more than 2^29 distinct words");
  Table nt{};
  if (int rc = alloc_table(nt, cap, g->stream)) {
    free_table(nt);
    return rc;
  }
  HIP_I(hipMemsetAsync(g->ctr + 1, 0, sizeof(unsigned long long), g->stream));
  hipLaunchKernelGGL(rehash_kernel, grid_for(g->cap), dim3(kBlock), 0, g->stream, g->tab, g->cap, nt, g->ctr + 1);
  HIP_I(hipGetLastError());
  unsigned long long f = 0;
  HIP_I(hipMemcpyAsync(&f, g->ctr + 1, sizeof(f), hipMemcpyDeviceToHost, g->stream));
  HIP_I(hipStreamSynchronize(g->stream));
  free_table(g->tab);
  g->tab = nt;
  g->cap = cap;
  if (f) return fail_i(W2V_ERR_STATE, "w2v_ingest_count: rehash lost words");
  return W2V_OK;
}

// hipcub's element counts are int: a chunk is at most INT32_MAX - 64 bytes
// (chunk_size_limit; the callers cut the file into such chunks), so its tokens
// (<= bytes / 2 + 1), tiles (<= bytes / 4096 + 2), the table (<= 2^30 slots,
// kMaxCap) and the words (<= 2^29) all fit the (int) casts below.
int ensure_work(w2v_ingest* g, int64_t bytes) {
  if (bytes < 0 || bytes > (int64_t)INT32_MAX - 64)
    return fail_i(W2V_ERR_UNSUPPORTED, "w2v_ingest: a chunk must be < 2^31 - 64 bytes (hipcub int counts)");
  if (g->work_cap >= bytes) return W2V_OK;
  dfree(g->buf); dfree(g->tile); dfree(g->starts); dfree(g->nl_after); dfree(g->slot); dfree(g->line_of);
  dfree(g->tok_id); dfree(g->kept); dfree(g->kpos); dfree(g->n_sel);
  if (g->temp) (void)hipFree(g->temp);
  g->temp = nullptr;
  g->work_cap = 0;
  const int64_t max_tok = bytes / 2 + 1;  // a token and its separator take >= 2 bytes
  HIP_I(hipMalloc(&g->buf, bytes + 1));
  const int64_t n_tiles = bytes / kTileBytes + 2;
  HIP_I(hipMalloc(&g->tile, n_tiles * sizeof(int64_t)));
  HIP_I(hipMalloc(&g->starts, max_tok * sizeof(int64_t)));
  HIP_I(hipMalloc(&g->nl_after, max_tok * sizeof(uint32_t)));
  HIP_I(hipMalloc(&g->slot, max_tok * sizeof(uint32_t)));
  HIP_I(hipMalloc(&g->line_of, max_tok * sizeof(int64_t)));
  HIP_I(hipMalloc(&g->tok_id, max_tok * sizeof(int32_t)));
  HIP_I(hipMalloc(&g->kept, max_tok * sizeof(int32_t)));
  HIP_I(hipMalloc(&g->kpos, max_tok * sizeof(int32_t)));
  HIP_I(hipMalloc(&g->n_sel, sizeof(int64_t)));
  // scratch for the selects and scans at the largest size
  size_t t1 = 0, t2 = 0, t3 = 0, t4 = 0;
  const int nk = (int)std::min<int64_t>(max_tok, INT32_MAX);
  HIP_I(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, g->tile, g->tile, (int)n_tiles));
  HIP_I(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, g->nl_after, g->line_of, nk));
  HIP_I(hipcub::DeviceSelect::If(nullptr, t3, g->tok_id, g->tok_id, g->n_sel, nk, NotNegative()));
  HIP_I(hipcub::DeviceScan::ExclusiveSum(nullptr, t4, g->kept, g->kpos, nk));
  g->temp_bytes = std::max({t1, t2, t3, t4});
  HIP_I(hipMalloc(&g->temp, g->temp_bytes));
  g->work_cap = bytes;
  return W2V_OK;
}

// The chunk's bytes on the device (copied unless the file is resident), and
// its token starts; returns the token count in *nt.
int tokenize(w2v_ingest* g, const char* data, int64_t off, int64_t n, int64_t* nt) {
  if (g->file) {
    g->cur = g->file + off;
  } else {
    HIP_I(hipMemcpyAsync(g->buf, data + off, n, hipMemcpyHostToDevice, g->stream));
    g->cur = g->buf;
  }
  const int64_t n_tiles = (n + kTileBytes - 1) / kTileBytes;
  if (n_tiles == 0) {
    *nt = 0;
    return W2V_OK;
  }
  HIP_I(hipMemsetAsync(g->tile + n_tiles, 0, sizeof(int64_t), g->stream));
  hipLaunchKernelGGL(tile_count_kernel, dim3((unsigned)n_tiles), dim3(256), 0, g->stream, g->cur, n, g->tile);
  HIP_I(hipGetLastError());
  size_t tb = g->temp_bytes;
  HIP_I(hipcub::DeviceScan::ExclusiveSum(g->temp, tb, g->tile, g->tile, (int)n_tiles + 1, g->stream));
  hipLaunchKernelGGL(tile_write_kernel, dim3((unsigned)n_tiles), dim3(256), 0, g->stream, g->cur, n, g->tile,
                     g->starts);
  HIP_I(hipGetLastError());
  HIP_I(hipMemcpyAsync(nt, g->tile + n_tiles, sizeof(int64_t), hipMemcpyDeviceToHost, g->stream));
  HIP_I(hipStreamSynchronize(g->stream));
  return W2V_OK;
}

// Line index of each token of the chunk (line_base + newlines before it in the
// chunk); returns the newline count after the chunk's last token in *after.
int lines_of(w2v_ingest* g, int64_t nt, int64_t line_base, int64_t* last_line, int64_t* after) {
  size_t tb = g->temp_bytes;
  HIP_I(hipcub::DeviceScan::ExclusiveSum(g->temp, tb, g->nl_after, g->line_of, (int)nt, g->stream));
  hipLaunchKernelGGL(add_base_kernel, grid_for(nt), dim3(kBlock), 0, g->stream, g->line_of, nt, line_base);
  HIP_I(hipGetLastError());
  uint32_t last_nl = 0;
  HIP_I(hipMemcpyAsync(last_line, g->line_of + nt - 1, sizeof(int64_t), hipMemcpyDeviceToHost, g->stream));
  HIP_I(hipMemcpyAsync(&last_nl, g->nl_after + nt - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, g->stream));
  HIP_I(hipStreamSynchronize(g->stream));
  *after = last_nl;
  return W2V_OK;
}

// Newlines before the chunk's first token (its leading whitespace).
int64_t leading_newlines(const char* p, int64_t n) {
  int64_t k = 0;
  for (int64_t i = 0; i < n && host_space(p[i]); ++i) k += p[i] == '\n';
  return k;
}

int64_t chunk_size_limit(const w2v_ingest* g) { return std::min<int64_t>(g->chunk, (int64_t)INT32_MAX - 64); }

// The used slots sorted by first occurrence -> g->order; their counts -> g->word_count.
int order_words(w2v_ingest* g, int64_t n_words) {
  dfree(g->order);
  HIP_I(hipMalloc(&g->order, std::max<int64_t>(n_words, 1) * sizeof(int64_t)));
  if (n_words == 0) return W2V_OK;
  int64_t* slots = nullptr;
  unsigned long long *firsts = nullptr, *firsts_sorted = nullptr;
  void* tmp = nullptr;
  auto cleanup = [&] {
    dfree(slots); dfree(firsts); dfree(firsts_sorted);
    if (tmp) (void)hipFree(tmp);
  };
  int rc = [&]() -> int {
    HIP_I(hipMalloc(&slots, n_words * sizeof(int64_t)));
    HIP_I(hipMalloc(&firsts, n_words * sizeof(unsigned long long)));
    HIP_I(hipMalloc(&firsts_sorted, n_words * sizeof(unsigned long long)));
    hipcub::CountingInputIterator<int64_t> it(0);
    size_t t1 = 0, t2 = 0;
    HIP_I(hipcub::DeviceSelect::If(nullptr, t1, it, slots, g->n_sel, (int)g->cap, UsedSlot{g->tab.key}, g->stream));
    HIP_I(hipcub::DeviceRadixSort::SortPairs(nullptr, t2, firsts, firsts_sorted, slots, g->order, (int)n_words, 0, 64,
                                             g->stream));
    const size_t tb = std::max<size_t>(std::max(t1, t2), 1);
    HIP_I(hipMalloc(&tmp, tb));
    size_t t = tb;
    HIP_I(hipcub::DeviceSelect::If(tmp, t, it, slots, g->n_sel, (int)g->cap, UsedSlot{g->tab.key}, g->stream));
    int64_t sel = 0;
    HIP_I(hipMemcpyAsync(&sel, g->n_sel, sizeof(int64_t), hipMemcpyDeviceToHost, g->stream));
    HIP_I(hipStreamSynchronize(g->stream));
    if (sel != n_words) return fail_i(W2V_ERR_STATE, "w2v_ingest_count: used-slot count mismatch");
    hipLaunchKernelGGL(gather_first_kernel, grid_for(n_words), dim3(kBlock), 0, g->stream, slots, n_words,
                       g->tab.first, firsts);
    HIP_I(hipGetLastError());
    t = tb;
    HIP_I(hipcub::DeviceRadixSort::SortPairs(tmp, t, firsts, firsts_sorted, slots, g->order, (int)n_words, 0, 64,
                                             g->stream));
    HIP_I(hipStreamSynchronize(g->stream));
    return W2V_OK;
  }();
  cleanup();
  return rc;
}

}  // namespace

extern "C" {

int w2v_ingest_create(int32_t device, int32_t format, int64_t chunk_bytes, w2v_ingest** out) {
  if (!out) return fail_i(W2V_ERR_ARG, "w2v_ingest_create: null argument");
  *out = nullptr;
  if (format != W2V_INGEST_LINES && format != W2V_INGEST_TEXT8) return fail_i(W2V_ERR_ARG, "bad ingest format");
  if (chunk_bytes < 0) return fail_i(W2V_ERR_ARG, "chunk_bytes must be >= 0");
  w2v_ingest* g = new w2v_ingest();
  g->format = format;
  if (chunk_bytes > 0) g->chunk = std::max<int64_t>(chunk_bytes, 1 << 12);
  hipError_t e = hipSuccess;
  if (device >= 0) g->device = device;
  else e = hipGetDevice(&g->device);
  if (e == hipSuccess) e = hipSetDevice(g->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&g->ctr, 3 * sizeof(unsigned long long));
  if (e != hipSuccess) {
    w2v_ingest_destroy(g);
    return fail_i(W2V_ERR_HIP, std::string("w2v_ingest_create: ") + hipGetErrorString(e));
  }
  *out = g;
  return W2V_OK;
}

void w2v_ingest_destroy(w2v_ingest* g) {
  if (!g) return;
  (void)hipSetDevice(g->device);
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  free_table(g->tab);
  dfree(g->ctr); dfree(g->order); dfree(g->ids); dfree(g->offsets); dfree(g->file);
  dfree(g->buf); dfree(g->tile); dfree(g->starts); dfree(g->nl_after); dfree(g->slot); dfree(g->line_of);
  dfree(g->tok_id); dfree(g->kept); dfree(g->kpos); dfree(g->n_sel);
  if (g->temp) (void)hipFree(g->temp);
  if (g->stream) (void)hipStreamDestroy(g->stream);
  delete g;
}

int w2v_ingest_set_resident(w2v_ingest* g, int64_t max_bytes) {
  if (!g) return fail_i(W2V_ERR_ARG, "null ingest");
  g->resident_max = max_bytes < 0 ? kResidentMax : max_bytes;
  return W2V_OK;
}

int w2v_ingest_count(w2v_ingest* g, const char* data, int64_t n) {
  if (!g || (n > 0 && !data) || n < 0) return fail_i(W2V_ERR_ARG, "w2v_ingest_count: bad argument");
  w2v::Range range_("w2v_ingest_count");
  HIP_I(hipSetDevice(g->device));
  g->counted = g->mapped = false;
  const bool lines = g->format == W2V_INGEST_LINES;
  const auto cs = chunks(data, n, chunk_size_limit(g), lines);
  int64_t biggest = 0;
  for (auto& c : cs) biggest = std::max(biggest, c.second - c.first);
  if (biggest > (int64_t)INT32_MAX - 64) return fail_i(W2V_ERR_UNSUPPORTED, "w2v_ingest_count: a line longer than 2 GiB");
  if (int rc = ensure_work(g, std::max<int64_t>(biggest, 1))) return rc;
  // a file that fits the residency budget crosses PCIe once: pass 2 reads this copy
  dfree(g->file);
  g->file_n = -1;
  // ... and only while it leaves at least half of the device's free memory to
  // the work buffers, the table and whatever trains next on this device
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
  if (n > 0 && n <= g->resident_max && (uint64_t)n <= (uint64_t)free_b / 2) {
    if (hipMalloc(&g->file, n) == hipSuccess) {
      HIP_I(hipMemcpyAsync(g->file, data, n, hipMemcpyHostToDevice, g->stream));
      g->file_n = n;
    } else {
      (void)hipGetLastError();  // no room: stream the chunks in both passes instead
      g->file = nullptr;
    }
  }
  // the table starts at 2^16..2^24 slots and doubles whenever it is half full
  free_table(g->tab);
  int64_t cap = (int64_t)1 << 16;
  while (cap < std::min<int64_t>(n / 64, (int64_t)1 << 24)) cap <<= 1;
  if (int rc = alloc_table(g->tab, cap, g->stream)) return rc;
  g->cap = cap;
  HIP_I(hipMemsetAsync(g->ctr, 0, 3 * sizeof(unsigned long long), g->stream));
  int64_t raw = 0, newlines = 0;
  for (auto& c : cs) {
    const int64_t len = c.second - c.first;
    int64_t nt = 0;
    if (int rc = tokenize(g, data, c.first, len, &nt)) return rc;
    newlines += leading_newlines(data + c.first, len);
    if (nt > 0) {
      for (;;) {  // insert until no token failed to find a slot and the table is at most half full
        HIP_I(hipMemsetAsync(g->ctr + 1, 0, sizeof(unsigned long long), g->stream));
        hipLaunchKernelGGL(insert_kernel, grid_for(nt), dim3(kBlock), 0, g->stream, g->cur, len, g->starts, nt,
                           c.first, g->tab, g->slot, g->nl_after, g->ctr, g->ctr + 1);
        HIP_I(hipGetLastError());
        unsigned long long cnt[2] = {0, 0};
        HIP_I(hipMemcpyAsync(cnt, g->ctr, sizeof(cnt), hipMemcpyDeviceToHost, g->stream));
        HIP_I(hipStreamSynchronize(g->stream));
        if (cnt[1] == 0 && (int64_t)cnt[0] * 2 <= g->cap) break;
        if (int rc = grow(g, (int64_t)cnt[0] + (int64_t)cnt[1])) return rc;
      }
      hipLaunchKernelGGL(count_kernel, grid_for(nt / 16), dim3(kBlock), 0, g->stream, g->slot, nt, g->tab.count);
      HIP_I(hipGetLastError());
      int64_t last_line = 0, after = 0;
      if (int rc = lines_of(g, nt, 0, &last_line, &after)) return rc;
      newlines += last_line + after;
    }
    raw += nt;
  }
  unsigned long long used = 0;
  HIP_I(hipMemcpy(&used, g->ctr, sizeof(used), hipMemcpyDeviceToHost));
  if (int rc = order_words(g, (int64_t)used)) return rc;
  g->n_words = (int64_t)used;
  g->word_count.assign((size_t)used, 0);
  if (used > 0) {
    int64_t *d_first = nullptr, *d_count = nullptr;
    int32_t* d_len = nullptr;
    HIP_I(hipMalloc(&d_first, used * sizeof(int64_t)));
    HIP_I(hipMalloc(&d_len, used * sizeof(int32_t)));
    HIP_I(hipMalloc(&d_count, used * sizeof(int64_t)));
    hipLaunchKernelGGL(gather_words_kernel, grid_for((int64_t)used), dim3(kBlock), 0, g->stream, g->order,
                       (int64_t)used, g->tab, d_first, d_len, d_count);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(g->word_count.data(), d_count, used * sizeof(int64_t), hipMemcpyDeviceToHost,
                                            g->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g->stream);
    dfree(d_first); dfree(d_len); dfree(d_count);
    if (e != hipSuccess) return fail_i(W2V_ERR_HIP, std::string("w2v_ingest_count: ") + hipGetErrorString(e));
  }
  g->n_bytes = n;
  g->raw_tokens = raw;
  // sentences: lines (getline: a final unterminated line counts when it holds bytes) or 1000-token cuts
  if (lines) g->n_sentences = newlines + ((n > 0 && data[n - 1] != '\n') ? 1 : 0);
  else g->n_sentences = (raw + kText8Sentence - 1) / kText8Sentence;
  g->counted = true;
  return W2V_OK;
}

int w2v_ingest_summary(w2v_ingest* g, int64_t* n_words, int64_t* raw_tokens, int64_t* n_sentences) {
  if (!g) return fail_i(W2V_ERR_ARG, "null ingest");
  if (!g->counted) return fail_i(W2V_ERR_STATE, "w2v_ingest_count first");
  if (n_words) *n_words = g->n_words;
  if (raw_tokens) *raw_tokens = g->raw_tokens;
  if (n_sentences) *n_sentences = g->n_sentences;
  return W2V_OK;
}

int w2v_ingest_words(w2v_ingest* g, int64_t* first_offset, int32_t* length, int64_t* count) {
  if (!g) return fail_i(W2V_ERR_ARG, "null ingest");
  if (!g->counted) return fail_i(W2V_ERR_STATE, "w2v_ingest_count first");
  const int64_t m = g->n_words;
  if (m == 0) return W2V_OK;
  HIP_I(hipSetDevice(g->device));
  int64_t *d_first = nullptr, *d_count = nullptr;
  int32_t* d_len = nullptr;
  auto cleanup = [&] { dfree(d_first); dfree(d_len); dfree(d_count); };
  int rc = [&]() -> int {
    HIP_I(hipMalloc(&d_first, m * sizeof(int64_t)));
    HIP_I(hipMalloc(&d_len, m * sizeof(int32_t)));
    HIP_I(hipMalloc(&d_count, m * sizeof(int64_t)));
    hipLaunchKernelGGL(gather_words_kernel, grid_for(m), dim3(kBlock), 0, g->stream, g->order, m, g->tab, d_first,
                       d_len, d_count);
    HIP_I(hipGetLastError());
    if (first_offset) HIP_I(hipMemcpyAsync(first_offset, d_first, m * sizeof(int64_t), hipMemcpyDeviceToHost, g->stream));
    if (length) HIP_I(hipMemcpyAsync(length, d_len, m * sizeof(int32_t), hipMemcpyDeviceToHost, g->stream));
    if (count) HIP_I(hipMemcpyAsync(count, d_count, m * sizeof(int64_t), hipMemcpyDeviceToHost, g->stream));
    HIP_I(hipStreamSynchronize(g->stream));
    return W2V_OK;
  }();
  cleanup();
  return rc;
}

int w2v_ingest_map(w2v_ingest* g, const char* data, int64_t n, const int32_t* vocab_index, int64_t n_words) {
  if (!g || (n > 0 && !data) || (n_words > 0 && !vocab_index)) return fail_i(W2V_ERR_ARG, "w2v_ingest_map: null argument");
  if (!g->counted) return fail_i(W2V_ERR_STATE, "w2v_ingest_count first");
  if (n != g->n_bytes || n_words != g->n_words) return fail_i(W2V_ERR_ARG, "w2v_ingest_map: not the counted corpus");
  w2v::Range range_("w2v_ingest_map");
  HIP_I(hipSetDevice(g->device));
  g->mapped = false;
  int32_t vmax = -1;
  for (int64_t k = 0; k < n_words; ++k) {
    if (vocab_index[k] < -1) return fail_i(W2V_ERR_ARG, "vocab_index entries must be >= -1");
    vmax = std::max(vmax, vocab_index[k]);
  }
  // per-id token histogram: every occurrence of an in-vocab word is kept
  g->hist.assign((size_t)vmax + 1, 0);
  for (int64_t k = 0; k < n_words; ++k)
    if (vocab_index[k] >= 0) g->hist[(size_t)vocab_index[k]] += g->word_count[(size_t)k];
  // slot -> vocab index
  int32_t *d_slot = nullptr, *d_vidx = nullptr;
  auto cleanup = [&] { dfree(d_slot); dfree(d_vidx); };
  int rc = [&]() -> int {
    HIP_I(hipMalloc(&d_slot, g->cap * sizeof(int32_t)));
    HIP_I(hipMemsetAsync(d_slot, 0xFF, g->cap * sizeof(int32_t), g->stream));
    if (n_words > 0) {
      HIP_I(hipMalloc(&d_vidx, n_words * sizeof(int32_t)));
      HIP_I(hipMemcpyAsync(d_vidx, vocab_index, n_words * sizeof(int32_t), hipMemcpyHostToDevice, g->stream));
      hipLaunchKernelGGL(scatter_ids_kernel, grid_for(n_words), dim3(kBlock), 0, g->stream, g->order, d_vidx, n_words,
                         d_slot);
      HIP_I(hipGetLastError());
    }
    dfree(g->ids); dfree(g->offsets);
    HIP_I(hipMalloc(&g->ids, std::max<int64_t>(g->raw_tokens, 1) * sizeof(int32_t)));
    HIP_I(hipMalloc(&g->offsets, (g->n_sentences + 1) * sizeof(int64_t)));
    HIP_I(hipMemsetAsync(g->offsets, 0, (g->n_sentences + 1) * sizeof(int64_t), g->stream));
    HIP_I(hipMemsetAsync(g->ctr + 2, 0, sizeof(unsigned long long), g->stream));
    const bool lines = g->format == W2V_INGEST_LINES;
    const auto cs = chunks(data, n, chunk_size_limit(g), lines);
    int64_t raw = 0, kept = 0, line_base = 0, prev_line = -1;
    for (auto& c : cs) {
      const int64_t len = c.second - c.first;
      int64_t nt = 0;
      if (int rc2 = tokenize(g, data, c.first, len, &nt)) return rc2;
      line_base += leading_newlines(data + c.first, len);
      if (nt > 0) {
        hipLaunchKernelGGL(map_kernel, grid_for(nt), dim3(kBlock), 0, g->stream, g->cur, len, g->starts, nt, g->tab,
                           d_slot, g->tok_id, g->kept, g->nl_after, g->ctr + 2);
        HIP_I(hipGetLastError());
        int64_t last_line = 0, after = 0;
        if (int rc2 = lines_of(g, nt, line_base, &last_line, &after)) return rc2;
        size_t tb = g->temp_bytes;
        HIP_I(hipcub::DeviceScan::ExclusiveSum(g->temp, tb, g->kept, g->kpos, (int)nt, g->stream));
        hipLaunchKernelGGL(boundary_kernel, grid_for(nt), dim3(kBlock), 0, g->stream, g->kpos, g->line_of, nt, raw, kept,
                           prev_line, lines ? 0 : 1, g->offsets);
        HIP_I(hipGetLastError());
        // append the chunk's in-vocab ids
        tb = g->temp_bytes;
        HIP_I(hipcub::DeviceSelect::If(g->temp, tb, g->tok_id, g->ids + kept, g->n_sel, (int)nt, NotNegative(),
                                       g->stream));
        int64_t sel = 0;
        HIP_I(hipMemcpyAsync(&sel, g->n_sel, sizeof(int64_t), hipMemcpyDeviceToHost, g->stream));
        HIP_I(hipStreamSynchronize(g->stream));
        kept += sel;
        prev_line = last_line;
        line_base = last_line + after;
      }
      raw += nt;
    }
    if (raw != g->raw_tokens) return fail_i(W2V_ERR_STATE, "w2v_ingest_map: token count differs from pass 1");
    // the sentences after the last token's (lines: trailing empty lines) and the end
    const int64_t tail = lines ? prev_line + 1 : g->n_sentences;
    hipLaunchKernelGGL(fill_kernel, grid_for(g->n_sentences + 1 - tail), dim3(kBlock), 0, g->stream, g->offsets, tail,
                       g->n_sentences + 1, kept);
    HIP_I(hipGetLastError());
    unsigned long long mism = 0;
    HIP_I(hipMemcpyAsync(&mism, g->ctr + 2, sizeof(mism), hipMemcpyDeviceToHost, g->stream));
    HIP_I(hipStreamSynchronize(g->stream));
    if (mism > 0)
      return fail_i(W2V_ERR_UNSUPPORTED, "w2v_ingest_map: " + std::to_string(mism) +
                                             " tokens matched a word by the first hash but not the second "
                                             "(a collision) or were not counted: the bytes differ from pass 1");
    g->n_ids = kept;
    return W2V_OK;
  }();
  cleanup();
  if (rc == W2V_OK) g->mapped = true;
  return rc;
}

int w2v_ingest_samples_size(w2v_ingest* g, int64_t* n_ids, int64_t* n_sentences, int64_t* train_words) {
  if (!g) return fail_i(W2V_ERR_ARG, "null ingest");
  if (!g->mapped) return fail_i(W2V_ERR_STATE, "w2v_ingest_map first");
  if (n_ids) *n_ids = g->n_ids;
  if (n_sentences) *n_sentences = g->n_sentences;
  if (train_words) *train_words = g->raw_tokens;
  return W2V_OK;
}

int w2v_ingest_download(w2v_ingest* g, int32_t* ids, int64_t* offsets) {
  if (!g) return fail_i(W2V_ERR_ARG, "null ingest");
  if (!g->mapped) return fail_i(W2V_ERR_STATE, "w2v_ingest_map first");
  HIP_I(hipSetDevice(g->device));
  if (ids && g->n_ids > 0) HIP_I(hipMemcpy(ids, g->ids, g->n_ids * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (offsets) HIP_I(hipMemcpy(offsets, g->offsets, (g->n_sentences + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
  return W2V_OK;
}

}  // extern "C"

namespace w2v {
IngestView ingest_view(const w2v_ingest* g) {
  IngestView v{};
  if (!g || !g->mapped) return v;
  v.device = g->device;
  v.ids = g->ids;
  v.n_ids = g->n_ids;
  v.offsets = g->offsets;
  v.n_sentences = g->n_sentences;
  v.train_words = g->raw_tokens;
  v.hist = g->hist.data();
  v.n_vocab = (int64_t)g->hist.size();
  v.ok = true;
  return v;
}
}  // namespace w2v
