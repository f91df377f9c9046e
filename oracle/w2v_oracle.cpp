// ============================================================================
// oracle/w2v_oracle.cpp — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
//
// A sequential CPU restatement of the reference's Word2Vec training path
// (lache/word2vec, /root/reference/Word2Vec.cpp), used only by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
// Nothing under word2vec_amd/ links or loads this file.
//
// Parity status: the reference itself is UNBUILDABLE in this image (it needs
// Eigen, which is absent; building it against a hand-written stand-in header is
// not allowed), and it ships no tests or fixtures. So this restatement is
// pinned (a) against libstdc++ 11.4 itself for every third-party behaviour the
// reference delegates to it (mt19937, uniform_int/real distributions,
// std::shuffle, heap ops, std::sort, unordered_map iteration) — see
// tests/golden/gen_libstdcxx_golden.cpp — and (b) against an independent
// numpy restatement of the float arithmetic (tests/test_oracle.py). The Eigen
// dot product is restated as a sequential fp32 sum (the north star's
// "sequential fp32 update"); Eigen's vectorised summation order is unpinned.
//
// Three draw modes share one trainer:
//   REF     — one shared std::mt19937, consumed exactly in the reference's
//             order; optionally records every draw (the replay stream).
//   REPLAY  — consumes a recorded stream instead of the generator.
//   PHILOX  — counter-based Philox4x32-10 draws keyed by (epoch, sentence,
//             position, slot, k): the device's throughput-mode RNG, restated
//             here independently so the HIP kernel can be checked bit-for-bit
//             on its RNG and within 1e-5 on its arithmetic.
// Build: oracle/Makefile (g++ -O2, no fast-math: see SURVEY.md §8(c)).
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <numeric>
#include <random>
#include <set>
#include <sstream>
#include <string>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct OrcCfg {
  int32_t iter, window, min_count, table_size, dim, negative;
  float subsample, init_alpha, min_alpha;
  int32_t cbow_mean, hs, cbow;
};

struct Orc {
  OrcCfg cfg;
  std::mt19937 gen;
  // corpus as strings (reference: vector<vector<string>>)
  std::vector<std::vector<std::string>> sentences;
  // vocab, in reference index order (Word2Vec.cpp:153-160)
  std::vector<std::string> words;
  std::vector<uint64_t> counts;
  std::vector<float> keep;  // Word::sample_probability
  std::unordered_map<std::string, int32_t> lookup;
  std::vector<std::vector<uint8_t>> codes;
  std::vector<std::vector<int32_t>> points;
  std::vector<uint32_t> table;
  // model (dense rows of `dim` floats)
  std::vector<float> W, C, S;  // S = synapses1
  std::vector<float> W0, C0, S0;  // snapshot taken right after train()'s init
  // samples (Word2Vec.cpp:212-230): token ids, OOV dropped
  std::vector<int32_t> ids;
  std::vector<int64_t> off;
  // recorded draws
  std::vector<uint32_t> stream;
  std::vector<int64_t> stream_off;  // [epoch * n_sent + sentence]
  std::vector<int64_t> orders;      // [epoch * n_sent + i]
  int64_t train_words = 0, current_words = 0;
  float last_alpha = 0.f;
  bool shared_negatives = false;  // sgsn_sentence instead of sg_sentence (configs[4])
};

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11) — restated independently of the device.
// ---------------------------------------------------------------------------
inline void philox4x32_10(const uint32_t ctr_in[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// libstdc++ generate_canonical<float,24> on one 32-bit draw (random.tcc:3348-3380)
inline float canonical_float(uint32_t x) {
  float r = (float)x / 4294967296.0f;
  if (r >= 1.0f) r = std::nextafter(1.0f, 0.0f);
  return r;
}

// ---------------------------------------------------------------------------
// Draw policies.
// ---------------------------------------------------------------------------
struct RefDraws {
  // One shared generator, reference order (Word2Vec.h:55-59, ctor :16-17).
  std::mt19937* g;
  std::uniform_real_distribution<float> uni{0.0f, 1.0f};
  std::uniform_int_distribution<int> win, tab;
  std::vector<uint32_t>* rec;
  static const bool kCanonicalTargets = false;
  RefDraws(std::mt19937* g_, int window, int table_size, std::vector<uint32_t>* rec_)
      : g(g_), win(0, window < 1 ? 0 : window - 1), tab(0, table_size - 1), rec(rec_) {}
  void at(int64_t, int64_t) {}
  void rebase(const uint32_t*) {}
  float uniform() {
    float u = uni(*g);
    if (rec) { uint32_t b; std::memcpy(&b, &u, 4); rec->push_back(b); }
    return u;
  }
  int window_shrink() {
    int r = win(*g);
    if (rec) rec->push_back((uint32_t)r);
    return r;
  }
  int table_pos(int, int) {
    int r = tab(*g);
    if (rec) rec->push_back((uint32_t)r);
    return r;
  }
};

struct ReplayDraws {
  const uint32_t* p;
  static const bool kCanonicalTargets = false;
  void at(int64_t, int64_t) {}
  void rebase(const uint32_t* q) { p = q; }
  float uniform() { float u; std::memcpy(&u, p++, 4); return u; }
  int window_shrink() { return (int)*p++; }
  int table_pos(int, int) { return (int)*p++; }
};

struct PhiloxDraws {
  uint32_t k0, k1, epoch;
  int window;
  int64_t table_size;
  uint32_t s, i;
  uint32_t tok[4];
  bool have_tok;
  static const bool kCanonicalTargets = true;
  void at(int64_t sent, int64_t pos) { s = (uint32_t)sent; i = (uint32_t)pos; have_tok = false; }
  void rebase(const uint32_t*) {}
  void token() {
    if (!have_tok) {
      uint32_t ctr[4] = {i, s, 0xFFFFFFFFu, epoch};
      philox4x32_10(ctr, k0, k1, tok);
      have_tok = true;
    }
  }
  float uniform() { token(); return canonical_float(tok[0]); }
  int window_shrink() {
    token();
    uint32_t w = (uint32_t)(window < 1 ? 1 : window);
    return (int)(((uint64_t)tok[1] * w) >> 32);
  }
  int table_pos(int slot, int k) {
    // k's low byte next to the slot, its high bits above the epoch (k < 256: the epoch alone)
    uint32_t ctr[4] = {i, s, ((uint32_t)slot << 8) | ((uint32_t)k & 255u), epoch ^ (((uint32_t)k >> 8) << 20)}, o[4];
    philox4x32_10(ctr, k0, k1, o);
    uint64_t x = ((uint64_t)o[1] << 32) | o[0];
    return (int)(uint64_t)(((unsigned __int128)x * (uint64_t)table_size) >> 64);
  }
};

// ---------------------------------------------------------------------------
// Vocabulary (Word2Vec.cpp:132-169), Huffman (:32-79), table (:81-113),
// subsampling (:115-130).
// ---------------------------------------------------------------------------
void orc_make_huffman(Orc& m) {
  const size_t V = m.words.size();
  m.codes.assign(V, {});
  m.points.assign(V, {});
  if (V < 2) return;
  // node n < V is leaf n; node V+i is the i-th merge.  (Word2Vec.cpp:46)
  std::vector<uint64_t> cnt(m.counts.begin(), m.counts.end());
  cnt.resize(2 * V - 1);
  std::vector<size_t> lchild(V - 1), rchild(V - 1);
  auto by_count = [&](size_t a, size_t b) { return cnt[a] > cnt[b]; };  // comp, :3-6
  std::vector<size_t> heap(V);
  std::iota(heap.begin(), heap.end(), 0);
  std::make_heap(heap.begin(), heap.end(), by_count);
  for (size_t i = 0; i + 1 < V; ++i) {
    std::pop_heap(heap.begin(), heap.end(), by_count);
    size_t a = heap.back(); heap.pop_back();
    std::pop_heap(heap.begin(), heap.end(), by_count);
    size_t b = heap.back(); heap.pop_back();
    cnt[V + i] = cnt[a] + cnt[b];
    lchild[i] = a; rchild[i] = b;
    heap.push_back(V + i);
    std::push_heap(heap.begin(), heap.end(), by_count);
  }
  // Depth-first walk with a LIFO list; right child popped first (:51-78).
  typedef std::tuple<size_t, std::vector<uint8_t>, std::vector<int32_t>> Item;
  std::list<Item> todo;
  todo.push_back(Item(heap[0], {}, {}));
  while (!todo.empty()) {
    Item it = todo.back();
    todo.pop_back();
    size_t node = std::get<0>(it);
    if (node < V) {
      m.codes[node] = std::get<1>(it);
      m.points[node] = std::get<2>(it);
      continue;
    }
    std::vector<uint8_t> c0 = std::get<1>(it), c1 = std::get<1>(it);
    c0.push_back(0); c1.push_back(1);
    std::vector<int32_t> p = std::get<2>(it);
    p.push_back((int32_t)(node - V));
    todo.push_back(Item(lchild[node - V], c0, p));
    todo.push_back(Item(rchild[node - V], c1, p));
  }
}

void orc_make_table(Orc& m) {
  const int ts = m.cfg.table_size;
  const size_t V = m.words.size();
  m.table.assign((size_t)ts, 0);
  std::vector<float> wr(V);
  float total = 0.0f;
  for (size_t i = 0; i < V; ++i) {
    wr[i] = std::pow((float)m.counts[i], 0.75f);  // float powf
    total += wr[i];
  }
  size_t w = 0;
  float cum = wr[0] / total;
  float edge = ts * cum;
  for (int i = 0; i < ts; ++i) {
    m.table[i] = (uint32_t)w;
    if (i > edge && w < V - 1) {  // int i promoted to float here
      cum += wr[++w] / total;
      edge = ts * cum;
    } else if (w == V - 1) {
      for (; i < ts; ++i) m.table[i] = (uint32_t)w;
      break;
    }
  }
}

void orc_make_keep(Orc& m) {
  const size_t V = m.words.size();
  long total = 0;
  for (size_t i = 0; i < V; ++i) total += (long)m.counts[i];
  const float thr = m.cfg.subsample * total;
  m.keep.assign(V, 1.0f);
  if (m.cfg.subsample > 0) {
    for (size_t i = 0; i < V; ++i) {
      float c = (float)m.counts[i];
      float p = (std::sqrt(c / thr) + 1) * thr / c;
      m.keep[i] = std::min(p, 1.0f);
    }
  }
}

void orc_build_vocab_impl(Orc& m) {
  std::unordered_map<std::string, int> tally;
  for (auto& sent : m.sentences)
    for (auto& w : sent) {
      if (tally.count(w) > 0) tally[w]++;
      else tally[w] = 1;
    }
  std::vector<std::pair<std::string, uint64_t>> kept;
  for (auto kv : tally)
    if (kv.second >= m.cfg.min_count) kept.push_back({kv.first, (uint64_t)kv.second});
  // std::sort over indices with the reference comparator (count desc); the
  // permutation depends only on comparison outcomes, so it equals sorting Word*.
  std::vector<size_t> perm(kept.size());
  std::iota(perm.begin(), perm.end(), 0);
  std::sort(perm.begin(), perm.end(),
            [&](size_t a, size_t b) { return kept[a].second > kept[b].second; });
  m.words.clear(); m.counts.clear(); m.lookup.clear();
  for (size_t i = 0; i < perm.size(); ++i) {
    m.words.push_back(kept[perm[i]].first);
    m.counts.push_back(kept[perm[i]].second);
    m.lookup[m.words.back()] = (int32_t)i;
  }
  if (m.cfg.hs) orc_make_huffman(m);
  if (m.cfg.negative) orc_make_table(m);
  orc_make_keep(m);
}

// init_weights (Word2Vec.cpp:198-210); cbow+hs random C is this build's
// documented deviation (the reference reads an unallocated C there).
void orc_init_weights_impl(Orc& m) {
  const size_t V = m.words.size(), d = (size_t)m.cfg.dim;
  std::uniform_real_distribution<float> dist(-0.5, 0.5);
  m.W.resize(V * d);
  for (size_t k = 0; k < V * d; ++k) m.W[k] = dist(m.gen);
  for (size_t k = 0; k < V * d; ++k) m.W[k] = m.W[k] / (float)d;
  m.S.clear(); m.C.clear();
  if (m.cfg.hs) m.S.assign((V > 0 ? V - 1 : 0) * d, 0.0f);
  if (m.cfg.cbow && m.cfg.hs) {
    m.C.resize(V * d);
    for (size_t k = 0; k < V * d; ++k) m.C[k] = dist(m.gen);
    for (size_t k = 0; k < V * d; ++k) m.C[k] = m.C[k] / (float)d;
  } else if (!m.cfg.hs || m.cfg.negative > 0) {
    m.C.assign(V * d, 0.0f);
  }
}

void orc_build_sample_impl(Orc& m) {
  m.ids.clear();
  m.off.assign(1, 0);
  m.train_words = 0;
  for (auto& sent : m.sentences) {
    m.train_words += (int64_t)sent.size();
    for (auto& w : sent) {
      auto it = m.lookup.find(w);
      if (it != m.lookup.end()) m.ids.push_back(it->second);
    }
    m.off.push_back((int64_t)m.ids.size());
  }
}

// ---------------------------------------------------------------------------
// The per-target update (Word2Vec.cpp:238-246 HS, :261-268 NS).
// ---------------------------------------------------------------------------
inline float row_dot(const float* a, const float* b, int d) {
  float s = 0.0f;
  for (int k = 0; k < d; ++k) s += a[k] * b[k];
  return s;
}


// HS walk (Word2Vec.cpp:232-249): f and g computed through double as there.
inline void hs_step(Orc& m, int word, const float* x, float* g, float alpha) {
  const int d = m.cfg.dim;
  const std::vector<uint8_t>& cd = m.codes[word];
  const std::vector<int32_t>& pt = m.points[word];
  for (size_t k = 0; k < cd.size(); ++k) {
    float* r = &m.S[(size_t)pt[k] * d];
    float f = row_dot(r, x, d);
    f = 1.0 / (1.0 + std::exp(-f));
    float gg = (1.0 - cd[k] - f) * alpha;
    for (int e = 0; e < d; ++e) g[e] += gg * r[e];
    for (int e = 0; e < d; ++e) r[e] += gg * x[e];
  }
}

// NS (Word2Vec.cpp:251-271). REF/REPLAY iterate the same unordered_map the
// reference builds; PHILOX uses the device's canonical order (positive first,
// then first occurrences of the negatives in draw order).
template <class D>
inline void ns_step(Orc& m, int word, const float* x, float* g, float* M, float alpha, D& dr,
                    int slot) {
  const int d = m.cfg.dim;
  std::vector<std::pair<size_t, int>> tg;
  if (D::kCanonicalTargets) {
    tg.push_back({(size_t)word, 1});
    for (int k = 0; k < m.cfg.negative; ++k) {
      size_t n = m.table[dr.table_pos(slot, k)];
      bool seen = false;
      for (auto& t : tg) seen = seen || (t.first == n);
      if (!seen) tg.push_back({n, 0});
    }
  } else {
    std::unordered_map<size_t, uint8_t> hm;
    for (int k = 0; k < m.cfg.negative; ++k) hm[m.table[dr.table_pos(slot, k)]] = 0;
    hm[(size_t)word] = 1;
    for (auto kv : hm) tg.push_back({kv.first, (int)kv.second});
  }
  for (auto& t : tg) {
    float* r = &M[t.first * d];
    float f = row_dot(r, x, d);
    f = 1.0 / (1 + std::exp(-f));
    float gg = (t.second - f) * alpha;
    for (int e = 0; e < d; ++e) g[e] += gg * r[e];
    for (int e = 0; e < d; ++e) r[e] += gg * x[e];
  }
}

// Skip-gram sentence (Word2Vec.cpp:319-353): the center's W row is the input,
// held fixed over the window; each context word is predicted.
template <class D>
void sg_sentence(Orc& m, const int32_t* sent, int len, float alpha, D& dr, int64_t sid) {
  const int d = m.cfg.dim, win = m.cfg.window;
  std::vector<float> x(d), g(d);
  for (int i = 0; i < len; ++i) {
    const int c = sent[i];
    dr.at(sid, i);
    std::fill(g.begin(), g.end(), 0.0f);
    std::copy(&m.W[(size_t)c * d], &m.W[(size_t)c * d] + d, x.begin());
    if (m.keep[c] < dr.uniform()) continue;
    const int rw = dr.window_shrink();
    const int lo = std::max(0, i - win + rw), hi = std::min(len, i + win + 1 - rw);
    int slot = 0;
    for (int j = lo; j < hi; ++j) {
      if (j == i) continue;
      if (m.cfg.hs) hs_step(m, sent[j], x.data(), g.data(), alpha);
      if (m.cfg.negative > 0) ns_step(m, sent[j], x.data(), g.data(), m.C.data(), alpha, dr, slot);
      ++slot;
    }
    float* wc = &m.W[(size_t)c * d];
    for (int e = 0; e < d; ++e) wc[e] += g[e];
  }
}

// CBOW sentence (Word2Vec.cpp:273-317): input = sum of C rows over the SET of
// context ids (ascending), divided by the positional count when cbow_mean.
template <class D>
void cbow_sentence(Orc& m, const int32_t* sent, int len, float alpha, D& dr, int64_t sid) {
  const int d = m.cfg.dim, win = m.cfg.window;
  std::vector<float> h(d), g(d);
  for (int i = 0; i < len; ++i) {
    const int c = sent[i];
    dr.at(sid, i);
    if (m.keep[c] < dr.uniform()) continue;
    const int rw = dr.window_shrink();
    const int lo = std::max(0, i - win + rw), hi = std::min(len, i + win + 1 - rw);
    const int n = hi - lo - 1;
    if (n <= 0) continue;
    std::fill(h.begin(), h.end(), 0.0f);
    std::fill(g.begin(), g.end(), 0.0f);
    std::set<size_t> ctx;
    for (int j = lo; j < hi; ++j)
      if (j != i) ctx.insert((size_t)sent[j]);
    for (size_t id : ctx)
      for (int e = 0; e < d; ++e) h[e] += m.C[id * d + e];
    if (m.cfg.cbow_mean)
      for (int e = 0; e < d; ++e) h[e] /= (float)n;
    if (m.cfg.hs) hs_step(m, c, h.data(), g.data(), alpha);
    if (m.cfg.negative > 0) ns_step(m, c, h.data(), g.data(), m.W.data(), alpha, dr, 0);
    if (m.cfg.cbow_mean)
      for (int e = 0; e < d; ++e) g[e] /= (float)n;
    for (size_t id : ctx)
      for (int e = 0; e < d; ++e) m.C[id * d + e] += g[e];
  }
}

// Shared-negatives minibatch skip-gram (BASELINE configs[4]; the formulation
// of Ji et al., "Parallelizing Word2Vec in Shared and Distributed Memory",
// 2016: pWord2Vec). NOT a reference function: the reference has no minibatch
// path. It keeps the reference's subsampling draw, window shrink, alpha
// schedule and NS arithmetic (Word2Vec.cpp:251-271, 319-353) but, as
// word2vec.c and pWord2Vec do, drops subsampled tokens from the sentence
// before forming windows (the reference keeps them as contexts, :332-347),
// and batches one window into a dense update:
//   inputs  u: the unique context ids of the window over the kept tokens (W
//              rows), multiplicity m_u
//   outputs t: the center word (label 1, C row) and `negative` draws shared by
//              the whole window (label 0; a draw equal to the center or to an
//              earlier draw is dropped — the set semantics of :253-257)
//   L[u][t] = W[u].C[t];  E[u][t] = m_u * (label_t - sigma(L)) * alpha
//   W[u] += sum_t E[u][t] C[t];  C[t] += sum_u E[u][t] W[u]   (pre-update rows)
// i.e. the simultaneous update of every (context, output) pair of the window,
// with the input/output roles of word2vec.c (context predicts center); the
// reference's own per-pair loop has them the other way round (:339-347),
// which gives the same pair set over a symmetric window.
template <class D>
void sgsn_sentence(Orc& m, const int32_t* sent, int len, float alpha, D& dr, int64_t sid) {
  const int d = m.cfg.dim, win = m.cfg.window, K = m.cfg.negative;
  struct Kept { int id, pos, rw; };
  std::vector<Kept> kept;
  for (int i = 0; i < len; ++i) {  // the per-token draws, in the reference's order (:331-335)
    const int c = sent[i];
    dr.at(sid, i);
    if (m.keep[c] < dr.uniform()) continue;
    kept.push_back({c, i, dr.window_shrink()});
  }
  const int nk = (int)kept.size();
  std::vector<int> in_id, in_m, out_id, out_lab;
  std::vector<float> E, dW, dC;
  for (int t = 0; t < nk; ++t) {
    const int c = kept[t].id, rw = kept[t].rw;
    const int lo = std::max(0, t - win + rw), hi = std::min(nk, t + win + 1 - rw);
    in_id.clear(); in_m.clear();
    for (int j = lo; j < hi; ++j) {
      if (j == t) continue;
      size_t u = 0;
      while (u < in_id.size() && in_id[u] != kept[j].id) ++u;
      if (u == in_id.size()) { in_id.push_back(kept[j].id); in_m.push_back(0); }
      in_m[u] += 1;
    }
    if (in_id.empty()) continue;
    dr.at(sid, kept[t].pos);
    out_id.assign(1, c);
    out_lab.assign(1, 1);
    for (int k = 0; k < K; ++k) {
      const int n = (int)m.table[dr.table_pos(0, k)];
      bool seen = false;
      for (int o : out_id) seen = seen || (o == n);
      if (!seen) { out_id.push_back(n); out_lab.push_back(0); }
    }
    const size_t M = in_id.size(), T = out_id.size();
    E.assign(M * T, 0.0f);
    for (size_t u = 0; u < M; ++u)
      for (size_t tt = 0; tt < T; ++tt) {
        float f = row_dot(&m.W[(size_t)in_id[u] * d], &m.C[(size_t)out_id[tt] * d], d);
        f = 1.0 / (1 + std::exp(-f));
        const float g = (out_lab[tt] - f) * alpha;
        E[u * T + tt] = (float)in_m[u] * g;
      }
    dW.assign(M * d, 0.0f);
    dC.assign(T * d, 0.0f);
    for (size_t u = 0; u < M; ++u)
      for (size_t tt = 0; tt < T; ++tt) {
        const float e = E[u * T + tt];
        const float* wr = &m.W[(size_t)in_id[u] * d];
        const float* cr = &m.C[(size_t)out_id[tt] * d];
        for (int k = 0; k < d; ++k) {
          dW[u * d + k] += e * cr[k];
          dC[tt * d + k] += e * wr[k];
        }
      }
    for (size_t u = 0; u < M; ++u)
      for (int k = 0; k < d; ++k) m.W[(size_t)in_id[u] * d + k] += dW[u * d + k];
    for (size_t tt = 0; tt < T; ++tt)
      for (int k = 0; k < d; ++k) m.C[(size_t)out_id[tt] * d + k] += dC[tt * d + k];
  }
}

// alpha schedule (Word2Vec.cpp:379-380)
inline float schedule(const Orc& m, int64_t cw) {
  return std::max(m.cfg.min_alpha,
                  float(m.cfg.init_alpha * (1.0 - 1.0 / m.cfg.iter * cw / m.train_words)));
}

// One epoch over `order` in sequence (the single-thread form of :375-394).
template <class D>
void run_epoch(Orc& m, const int64_t* order, D& dr, int64_t epoch, const int64_t* replay_off,
               const uint32_t* replay_base, std::vector<int64_t>* rec_off) {
  const int64_t n = (int64_t)m.off.size() - 1;
  float alpha = m.cfg.init_alpha;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = order[i];
    if (i % 10 == 0) alpha = schedule(m, m.current_words);
    if (rec_off) (*rec_off)[(size_t)(epoch * n + s)] = (int64_t)m.stream.size();
    if (replay_off) dr.rebase(replay_base + replay_off[epoch * n + s]);
    const int32_t* sent = m.ids.data() + m.off[s];
    const int len = (int)(m.off[s + 1] - m.off[s]);
    if (m.shared_negatives) sgsn_sentence(m, sent, len, alpha, dr, s);
    else if (m.cfg.cbow) cbow_sentence(m, sent, len, alpha, dr, s);
    else sg_sentence(m, sent, len, alpha, dr, s);
    m.current_words += len;
  }
  m.last_alpha = alpha;
}

Orc* H(void* h) { return static_cast<Orc*>(h); }

std::vector<float>& matrix(Orc& m, int which, int initial) {
  if (initial) return which == 0 ? m.W0 : which == 1 ? m.C0 : m.S0;
  return which == 0 ? m.W : which == 1 ? m.C : m.S;
}

}  // namespace

// ============================================================================
// C ABI used by tests/ and bench.py (ctypes). Test infrastructure only.
// ============================================================================
extern "C" {

void* orc_new(int32_t iter, int32_t window, int32_t min_count, int32_t table_size, int32_t dim,
              int32_t negative, float subsample, float init_alpha, float min_alpha,
              int32_t cbow_mean, int32_t hs, int32_t cbow) {
  Orc* m = new Orc();
  m->cfg = OrcCfg{iter, window, min_count, table_size, dim, negative,
                  subsample, init_alpha, min_alpha, cbow_mean, hs, cbow};
  return m;
}
void orc_free(void* h) { delete H(h); }
void orc_seed(void* h, uint32_t s) { H(h)->gen.seed(s); }

// Sentences = lines, tokens = whitespace-separated (as Word2Vec.cpp:19-30).
void orc_load_text(void* h, const char* text, int64_t n) {
  Orc& m = *H(h);
  m.sentences.clear();
  std::string all(text, (size_t)n);
  std::istringstream lines(all);
  std::string line;
  while (std::getline(lines, line)) {
    std::istringstream toks(line);
    std::vector<std::string> sent;
    std::string t;
    while (toks >> t) sent.push_back(t);
    m.sentences.push_back(sent);
  }
}

void orc_build_vocab(void* h) { orc_build_vocab_impl(*H(h)); }
int64_t orc_vocab_size(void* h) { return (int64_t)H(h)->words.size(); }
const char* orc_vocab_word(void* h, int64_t i) { return H(h)->words[(size_t)i].c_str(); }
void orc_vocab_counts(void* h, int64_t* out) {
  for (size_t i = 0; i < H(h)->counts.size(); ++i) out[i] = (int64_t)H(h)->counts[i];
}
void orc_sample_probs(void* h, float* out) {
  std::copy(H(h)->keep.begin(), H(h)->keep.end(), out);
}
int64_t orc_huffman_total(void* h) {
  int64_t t = 0;
  for (auto& c : H(h)->codes) t += (int64_t)c.size();
  return t;
}
void orc_huffman(void* h, uint8_t* codes, int32_t* points, int64_t* off) {
  Orc& m = *H(h);
  int64_t t = 0;
  off[0] = 0;
  for (size_t w = 0; w < m.codes.size(); ++w) {
    for (size_t k = 0; k < m.codes[w].size(); ++k) {
      codes[t] = m.codes[w][k];
      points[t] = m.points[w][k];
      ++t;
    }
    off[w + 1] = t;
  }
}
int64_t orc_table_size(void* h) { return (int64_t)H(h)->table.size(); }
void orc_table(void* h, uint32_t* out) { std::copy(H(h)->table.begin(), H(h)->table.end(), out); }
// First table index of each word (V+1 entries; monotone table), by scanning.
void orc_table_bounds(void* h, int64_t* out) {
  Orc& m = *H(h);
  const size_t V = m.words.size();
  std::fill(out, out + V + 1, (int64_t)m.table.size());
  for (size_t i = m.table.size(); i-- > 0;) out[m.table[i]] = (int64_t)i;
  for (size_t w = V; w-- > 0;)
    if (out[w] > out[w + 1]) out[w] = out[w + 1];
}

void orc_init_weights(void* h) { orc_init_weights_impl(*H(h)); }
int64_t orc_matrix_rows(void* h, int32_t which) {
  return (int64_t)matrix(*H(h), which, 0).size() / H(h)->cfg.dim;
}
void orc_get_matrix(void* h, int32_t which, int32_t initial, float* out) {
  std::vector<float>& v = matrix(*H(h), which, initial);
  std::copy(v.begin(), v.end(), out);
}
void orc_set_matrix(void* h, int32_t which, const float* in, int64_t rows) {
  std::vector<float>& v = matrix(*H(h), which, 0);
  v.assign(in, in + rows * H(h)->cfg.dim);
}

void orc_build_sample(void* h) { orc_build_sample_impl(*H(h)); }
int64_t orc_n_tokens(void* h) { return (int64_t)H(h)->ids.size(); }
int64_t orc_n_sentences(void* h) { return (int64_t)H(h)->off.size() - 1; }
void orc_samples(void* h, int32_t* ids, int64_t* off) {
  std::copy(H(h)->ids.begin(), H(h)->ids.end(), ids);
  std::copy(H(h)->off.begin(), H(h)->off.end(), off);
}
int64_t orc_train_words(void* h) { return H(h)->train_words; }
int64_t orc_current_words(void* h) { return H(h)->current_words; }
float orc_last_alpha(void* h) { return H(h)->last_alpha; }

// The reference's train() (Word2Vec.cpp:356-396) run on one thread with the
// shared generator: init_weights again, build_sample, per epoch std::shuffle
// then the sentence loop. record != 0 keeps every draw and the orders.
void orc_train(void* h, int32_t record) {
  Orc& m = *H(h);
  orc_init_weights_impl(m);
  m.W0 = m.W; m.C0 = m.C; m.S0 = m.S;
  orc_build_sample_impl(m);
  m.current_words = 0;
  const int64_t n = (int64_t)m.off.size() - 1;
  std::vector<long> idx((size_t)n);
  std::iota(idx.begin(), idx.end(), 0);
  m.stream.clear();
  m.stream_off.assign((size_t)(n * m.cfg.iter), 0);
  m.orders.assign((size_t)(n * m.cfg.iter), 0);
  RefDraws dr(&m.gen, m.cfg.window, m.cfg.table_size, record ? &m.stream : nullptr);
  for (int it = 0; it < m.cfg.iter; ++it) {
    std::shuffle(idx.begin(), idx.end(), m.gen);
    std::vector<int64_t> ord(idx.begin(), idx.end());
    std::copy(ord.begin(), ord.end(), m.orders.begin() + it * n);
    run_epoch(m, ord.data(), dr, it, nullptr, nullptr, record ? &m.stream_off : nullptr);
  }
}
int64_t orc_stream_size(void* h) { return (int64_t)H(h)->stream.size(); }
void orc_stream(void* h, uint32_t* s, int64_t* off, int64_t* orders) {
  Orc& m = *H(h);
  std::copy(m.stream.begin(), m.stream.end(), s);
  std::copy(m.stream_off.begin(), m.stream_off.end(), off);
  std::copy(m.orders.begin(), m.orders.end(), orders);
}

// Train `epochs` epochs from the CURRENT matrices with a given per-epoch order
// (n_sent per epoch), drawing from a recorded stream (replay) or Philox.
// current_words continues from `cw0`; train_words must be set (build_sample).
void orc_train_replay(void* h, int32_t epochs, const int64_t* orders, const uint32_t* stream,
                      const int64_t* stream_off, int64_t cw0) {
  Orc& m = *H(h);
  const int64_t n = (int64_t)m.off.size() - 1;
  m.current_words = cw0;
  ReplayDraws dr{stream};
  for (int e = 0; e < epochs; ++e) run_epoch(m, orders + e * n, dr, e, stream_off, stream, nullptr);
}
void orc_train_philox(void* h, int32_t epoch0, int32_t epochs, const int64_t* orders,
                      uint64_t key, int64_t cw0) {
  Orc& m = *H(h);
  const int64_t n = (int64_t)m.off.size() - 1;
  m.current_words = cw0;
  PhiloxDraws dr;
  dr.k0 = (uint32_t)key; dr.k1 = (uint32_t)(key >> 32);
  dr.window = m.cfg.window; dr.table_size = m.cfg.table_size;
  for (int e = 0; e < epochs; ++e) {
    dr.epoch = (uint32_t)(epoch0 + e);
    run_epoch(m, orders + e * n, dr, epoch0 + e, nullptr, nullptr, nullptr);
  }
}

// The reference's OpenMP epoch (Word2Vec.cpp:375-394) on `threads` threads
// over a given order, with the Philox draws: `#pragma omp parallel for` with
// the default (static) schedule, so thread t walks the t-th contiguous block
// of the order; alpha refreshed every 10th index from the shared word counter
// (:379-380) and the counter bumped atomically (:392-393); the matrices are
// updated without synchronisation (the reference's Hogwild). The Philox draws
// are keyed by (epoch, sentence, position), so this differs from
// orc_train_philox ONLY by the threads' concurrency: the anchor of what the
// reference's own parallel loop does to the vectors.
void orc_train_philox_omp(void* h, int32_t threads, int32_t epoch0, int32_t epochs, const int64_t* orders,
                          uint64_t key, int64_t cw0) {
  Orc& m = *H(h);
  const int64_t n = (int64_t)m.off.size() - 1;
  int64_t cw = cw0;
  float alpha = m.cfg.init_alpha;
#ifdef _OPENMP
  omp_set_num_threads(threads);
#else
  (void)threads;
#endif
  for (int e = 0; e < epochs; ++e) {
    const int64_t* order = orders + (int64_t)e * n;
#pragma omp parallel
    {
      PhiloxDraws dr;
      dr.k0 = (uint32_t)key; dr.k1 = (uint32_t)(key >> 32);
      dr.window = m.cfg.window; dr.table_size = m.cfg.table_size;
      dr.epoch = (uint32_t)(epoch0 + e);
#pragma omp for schedule(static)
      for (int64_t i = 0; i < n; ++i) {
        if (i % 10 == 0) {
          int64_t snap;
#pragma omp atomic read
          snap = cw;
          float a = schedule(m, snap);
#pragma omp atomic write
          alpha = a;
        }
        float a_now;
#pragma omp atomic read
        a_now = alpha;
        const int64_t s = order[i];
        const int32_t* sent = m.ids.data() + m.off[s];
        const int len = (int)(m.off[s + 1] - m.off[s]);
        if (m.shared_negatives) sgsn_sentence(m, sent, len, a_now, dr, s);
        else if (m.cfg.cbow) cbow_sentence(m, sent, len, a_now, dr, s);
        else sg_sentence(m, sent, len, a_now, dr, s);
#pragma omp atomic
        cw += len;
      }
    }
  }
  m.current_words = cw;
  m.last_alpha = alpha;
}

// Shared-negatives minibatch skip-gram (sgsn_sentence) for every later training call.
void orc_set_shared_negatives(void* h, int32_t on) { H(h)->shared_negatives = on != 0; }

void orc_philox(const uint32_t* ctr, uint64_t key, uint32_t* out) {
  philox4x32_10(ctr, (uint32_t)key, (uint32_t)(key >> 32), out);
}

// CPU baseline timing leg (bench.py cpu_baseline): the reference's OpenMP loop
// (:375-394) with its per-call hash map / set, static schedule and shared
// alpha, but one generator per thread (the shared one is a data race, UB).
// Trains `n_sent_limit` sentences (a bounded sample) from the current model.
// Returns the in-vocab words consumed.
int64_t orc_train_omp_shared(void* h, int32_t threads, int64_t n_sent_limit, uint32_t seed, int32_t shared_rng);
int64_t orc_train_omp(void* h, int32_t threads, int64_t n_sent_limit, uint32_t seed) {
  return orc_train_omp_shared(h, threads, n_sent_limit, seed, 0);
}
// shared_rng != 0: every thread draws from ONE mt19937, unsynchronised, as the
// reference does (Word2Vec.h:56 `generator`, used by all OpenMP threads at
// Word2Vec.cpp:255,282,285,332,335 — a data race, undefined behaviour; kept
// because it is what the reference build runs and times).
int64_t orc_train_omp_shared(void* h, int32_t threads, int64_t n_sent_limit, uint32_t seed, int32_t shared_rng) {
  Orc& m = *H(h);
  std::mt19937 shared_gen(seed);
  const int64_t n = std::min<int64_t>((int64_t)m.off.size() - 1, n_sent_limit);
  int64_t cw = 0;
  float alpha = m.cfg.init_alpha;
#ifdef _OPENMP
  omp_set_num_threads(threads);
#else
  (void)threads;
#endif
#pragma omp parallel
  {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    std::mt19937 g(seed + 7919u * (uint32_t)tid);
    RefDraws dr(shared_rng ? &shared_gen : &g, m.cfg.window, m.cfg.table_size, nullptr);
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      if (i % 10 == 0) {
        int64_t snap;
#pragma omp atomic read
        snap = cw;
        float a = schedule(m, snap);
#pragma omp atomic write
        alpha = a;
      }
      float a_now;
#pragma omp atomic read
      a_now = alpha;
      const int32_t* sent = m.ids.data() + m.off[i];
      const int len = (int)(m.off[i + 1] - m.off[i]);
      if (m.shared_negatives) sgsn_sentence(m, sent, len, a_now, dr, i);
      else if (m.cfg.cbow) cbow_sentence(m, sent, len, a_now, dr, i);
      else sg_sentence(m, sent, len, a_now, dr, i);
#pragma omp atomic
      cw += len;
    }
  }
  return cw;
}

// Direct ids/vocab injection (bench path: synthetic Zipf ids, no strings).
// counts must already be in reference order (descending).
void orc_set_vocab_counts(void* h, const int64_t* counts, int64_t V) {
  Orc& m = *H(h);
  m.words.clear(); m.counts.clear(); m.lookup.clear();
  for (int64_t i = 0; i < V; ++i) {
    m.words.push_back("w" + std::to_string(i));
    m.counts.push_back((uint64_t)counts[i]);
  }
  if (m.cfg.hs) orc_make_huffman(m);
  if (m.cfg.negative) orc_make_table(m);
  orc_make_keep(m);
}
void orc_set_samples(void* h, const int32_t* ids, const int64_t* off, int64_t n_sent,
                     int64_t train_words) {
  Orc& m = *H(h);
  m.off.assign(off, off + n_sent + 1);
  m.ids.assign(ids, ids + off[n_sent]);
  m.train_words = train_words;
}

// The public per-call methods (Word2Vec.h:81-84) on the oracle's generator.
void orc_train_sentence(void* h, const int32_t* ids, int64_t n, float alpha, int32_t cbow) {
  Orc& m = *H(h);
  RefDraws dr(&m.gen, m.cfg.window, m.cfg.table_size, nullptr);
  if (cbow) cbow_sentence(m, ids, (int)n, alpha, dr, 0);
  else sg_sentence(m, ids, (int)n, alpha, dr, 0);
}
void orc_negative_sampling(void* h, int64_t word, const float* x, float* grad, int32_t which, float alpha) {
  Orc& m = *H(h);
  RefDraws dr(&m.gen, m.cfg.window, m.cfg.table_size, nullptr);
  ns_step(m, (int)word, x, grad, which == 0 ? m.W.data() : m.C.data(), alpha, dr, 0);
}
void orc_hierarchical_softmax(void* h, int64_t word, const float* x, float* grad, float alpha) {
  hs_step(*H(h), (int)word, x, grad, alpha);
}

}  // extern "C"
