// Host-side products of build_vocab consumed by the device hot path.
// Bit-exact restatements (see include/w2v_host.h); compiled with
// -ffp-contract=off and no fast-math so float rounding matches the reference's
// x86-64 -O2 build.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "w2v_host.h"

namespace w2vh {

// precalc_sampling (Word2Vec.cpp:115-130): thr = t * N in float (N = in-vocab
// total as long), p = min(float((sqrt(c/thr) + 1) * thr / c), 1).
void sample_probs(const int64_t* counts, int64_t V, float t, float* out) {
  long total = 0;
  for (int64_t i = 0; i < V; ++i) total += (long)counts[i];
  const float thr = t * total;
  for (int64_t i = 0; i < V; ++i) {
    if (!(t > 0)) {
      out[i] = 1.0f;
      continue;
    }
    const float c = (float)(uint64_t)counts[i];
    const float p = (std::sqrt(c / thr) + 1) * thr / c;
    out[i] = std::min(p, 1.0f);
  }
}

// make_table (Word2Vec.cpp:81-113) without materialising it. The loop writes
// word w at i and advances w right after the first i with (float)i > edge_w,
// so word w+1 starts at i+1; the last word fills the rest.
void table_bounds(const int64_t* counts, int64_t V, int32_t ts, int64_t* out) {
  std::vector<float> wr((size_t)V);
  float total = 0.0f;
  for (int64_t i = 0; i < V; ++i) {
    wr[(size_t)i] = std::pow((float)(uint64_t)counts[i], 0.75f);
    total += wr[(size_t)i];
  }
  out[0] = 0;
  float cum = wr[0] / total;
  float edge = ts * cum;
  int64_t w = 0;
  int64_t i = 0;  // next table index to be written
  while (w < V - 1 && i < ts) {
    // smallest j >= i with (float)j > edge; j < ts
    int64_t j = i;
    if (edge >= 0.0f && (double)edge > (double)j) {
      const double fl = std::floor((double)edge);
      if (fl > (double)j) j = (int64_t)fl;
    }
    while (j < ts && !((float)(int32_t)j > edge)) ++j;
    if (j >= ts) break;
    ++w;
    out[w] = j + 1;
    cum += wr[(size_t)w] / total;
    edge = ts * cum;
    i = j + 1;
  }
  // words the loop never reached have empty ranges at the end
  for (int64_t k = w + 1; k <= V; ++k) out[k] = ts;
}

void table_fill(const int64_t* b, int64_t V, uint32_t* t, int64_t n) {
  for (int64_t w = 0; w < V; ++w) {
    const int64_t lo = std::min<int64_t>(b[w], n), hi = std::min<int64_t>(b[w + 1], n);
    for (int64_t k = lo; k < hi; ++k) t[k] = (uint32_t)w;
  }
}

// create_huffman_tree (Word2Vec.cpp:32-79). The merge order must be the
// reference's, so the same libstdc++ heap algorithms run with the same
// comparator over the same initial sequence; the paths are then read
// bottom-up from parent links (a leaf's code/point sequence is fixed by the
// tree, not by the reference's traversal order).
int64_t huffman(const int64_t* counts, int64_t V, uint8_t* codes, int32_t* points, int64_t* off,
                int64_t cap) {
  if (V < 2) return -1;
  const size_t n = (size_t)V;
  std::vector<uint64_t> cnt(2 * n - 1);
  for (size_t k = 0; k < n; ++k) cnt[k] = (uint64_t)counts[k];
  std::vector<int64_t> parent(2 * n - 1, -1);
  std::vector<uint8_t> branch(2 * n - 1, 0);
  std::vector<size_t> heap(n);
  for (size_t k = 0; k < n; ++k) heap[k] = k;
  auto cmp = [&cnt](size_t a, size_t b) { return cnt[a] > cnt[b]; };
  std::make_heap(heap.begin(), heap.end(), cmp);
  for (size_t m = 0; m + 1 < n; ++m) {
    std::pop_heap(heap.begin(), heap.end(), cmp);
    const size_t l = heap.back();
    heap.pop_back();
    std::pop_heap(heap.begin(), heap.end(), cmp);
    const size_t r = heap.back();
    heap.pop_back();
    const size_t node = n + m;
    cnt[node] = cnt[l] + cnt[r];
    parent[l] = (int64_t)node; branch[l] = 0;
    parent[r] = (int64_t)node; branch[r] = 1;
    heap.push_back(node);
    std::push_heap(heap.begin(), heap.end(), cmp);
  }
  // path lengths
  std::vector<int32_t> depth(2 * n - 1, 0);
  for (size_t node = 2 * n - 2; node-- > 0;)  // parents have larger ids
    if (parent[node] >= 0) depth[node] = depth[(size_t)parent[node]] + 1;
  off[0] = 0;
  for (size_t k = 0; k < n; ++k) off[k + 1] = off[k] + depth[k];
  const int64_t total = off[n];
  if (cap < total || !codes || !points) return total;
  for (size_t k = 0; k < n; ++k) {
    int64_t pos = off[k + 1];
    size_t node = k;
    while (parent[node] >= 0) {
      --pos;
      codes[pos] = branch[node];
      points[pos] = (int32_t)((size_t)parent[node] - n);
      node = (size_t)parent[node];
    }
  }
  return total;
}

}  // namespace w2vh

extern "C" {

const char* w2v_host_version(void) { return "word2vec_amd-host 0.1"; }

void w2v_host_sample_probs(const int64_t* counts, int64_t V, float t, float* out) {
  w2vh::sample_probs(counts, V, t, out);
}
void w2v_host_table_bounds(const int64_t* counts, int64_t V, int32_t ts, int64_t* out) {
  w2vh::table_bounds(counts, V, ts, out);
}
void w2v_host_table_fill(const int64_t* b, int64_t V, uint32_t* t, int64_t n) {
  w2vh::table_fill(b, V, t, n);
}
int64_t w2v_host_huffman(const int64_t* counts, int64_t V, uint8_t* codes, int32_t* points,
                         int64_t* off, int64_t cap) {
  return w2vh::huffman(counts, V, codes, points, off, cap);
}

}  // extern "C"
