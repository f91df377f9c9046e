// Golden vectors from libstdc++ itself — the third-party library the reference
// delegates its randomness, heap, sort and hash-map behaviour to
// (Word2Vec.h:55-59; Word2Vec.cpp:16-17,37-48,143-155,200-203,253-259,282,285,
// 332,335,373). The reference cannot be built here (Eigen is absent), so these
// outputs of the real dependency pin the oracle and the device-side
// restatements (canonical float, Lemire downscale, shuffle, heap merge order,
// hash-map iteration order).
//
// Build+run (container, g++ 11.4 / libstdc++ 11.4):
//   g++ -std=c++11 -O2 tests/golden/gen_libstdcxx_golden.cpp -o /tmp/gen && /tmp/gen > tests/golden/libstdcxx_golden.json
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <list>
#include <numeric>
#include <random>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

static void arr_u64(const char* name, const std::vector<uint64_t>& v, bool last = false) {
  std::printf("\"%s\": [", name);
  for (size_t i = 0; i < v.size(); ++i) std::printf("%s%llu", i ? "," : "", (unsigned long long)v[i]);
  std::printf("]%s\n", last ? "" : ",");
}

// The reference's Huffman build, restated over pointer-to-node objects exactly
// as Word2Vec.cpp:32-79 uses them (heap of Word*, comp on count, DFS list).
struct Node {
  size_t index, count;
  Node *left, *right;
  std::vector<size_t> codes, points;
};
static bool node_comp(Node* a, Node* b) { return a->count > b->count; }

static void huffman_golden(const std::vector<size_t>& counts, std::vector<uint64_t>& codes,
                           std::vector<uint64_t>& points, std::vector<uint64_t>& off) {
  const size_t V = counts.size();
  std::vector<Node*> vocab;
  for (size_t i = 0; i < V; ++i) vocab.push_back(new Node{i, counts[i], nullptr, nullptr, {}, {}});
  std::vector<Node*> heap = vocab;
  std::make_heap(heap.begin(), heap.end(), node_comp);
  for (size_t i = 0; i < V - 1; ++i) {
    std::pop_heap(heap.begin(), heap.end(), node_comp);
    Node* a = heap.back(); heap.pop_back();
    std::pop_heap(heap.begin(), heap.end(), node_comp);
    Node* b = heap.back(); heap.pop_back();
    Node* w = new Node{i + V, a->count + b->count, a, b, {}, {}};
    heap.push_back(w);
    std::push_heap(heap.begin(), heap.end(), node_comp);
  }
  std::list<std::tuple<Node*, std::vector<size_t>, std::vector<size_t>>> st;
  st.push_back(std::make_tuple(heap[0], std::vector<size_t>(), std::vector<size_t>()));
  while (!st.empty()) {
    auto n = st.back(); st.pop_back();
    Node* nw = std::get<0>(n);
    if (nw->index < V) { nw->codes = std::get<1>(n); nw->points = std::get<2>(n); continue; }
    auto cl = std::get<1>(n), cr = cl;
    cl.push_back(0); cr.push_back(1);
    auto p = std::get<2>(n);
    p.push_back(nw->index - V);
    st.push_back(std::make_tuple(nw->left, cl, p));
    st.push_back(std::make_tuple(nw->right, cr, p));
  }
  off.assign(1, 0);
  for (size_t i = 0; i < V; ++i) {
    for (size_t k = 0; k < vocab[i]->codes.size(); ++k) {
      codes.push_back(vocab[i]->codes[k]);
      points.push_back(vocab[i]->points[k]);
    }
    off.push_back(codes.size());
  }
}

int main() {
  std::printf("{\n\"generator\": \"libstdc++ %d (g++ %d.%d)\",\n", (int)_GLIBCXX_RELEASE, __GNUC__, __GNUC_MINOR__);
  {  // raw mt19937 (Word2Vec.h:56)
    std::mt19937 g(1234);
    std::vector<uint64_t> v;
    for (int i = 0; i < 2000; ++i) v.push_back(g());
    arr_u64("mt19937_seed1234", v);
  }
  {  // uniform_real_distribution<float>(0,1) (uni_dis, Word2Vec.cpp:17) as float bits
    std::mt19937 g(77);
    std::uniform_real_distribution<float> d(0.0, 1.0);
    std::vector<uint64_t> v;
    for (int i = 0; i < 2000; ++i) { float f = d(g); uint32_t b; std::memcpy(&b, &f, 4); v.push_back(b); }
    arr_u64("uniform01_seed77_bits", v);
  }
  {  // init_weights' distribution (-0.5, 0.5) then /dim (Word2Vec.cpp:200-204), dim 7
    std::mt19937 g(5);
    std::uniform_real_distribution<float> d(-0.5, 0.5);
    std::vector<uint64_t> v;
    for (int i = 0; i < 700; ++i) { float f = d(g) / (float)7; uint32_t b; std::memcpy(&b, &f, 4); v.push_back(b); }
    arr_u64("init_weights_seed5_dim7_bits", v);
  }
  {  // distribution_window (0, window-1) and distribution_table (0, 1e8-1) (Word2Vec.cpp:17)
    std::mt19937 g(99);
    std::uniform_int_distribution<int> w(0, 4), t(0, 100000000 - 1);
    std::vector<uint64_t> a, b, c;
    for (int i = 0; i < 2000; ++i) a.push_back((uint64_t)w(g));
    for (int i = 0; i < 2000; ++i) b.push_back((uint64_t)t(g));
    std::mt19937 g2(99);
    for (int i = 0; i < 4000; ++i) c.push_back(g2());
    arr_u64("window5_seed99", a);
    arr_u64("table1e8_after_window_seed99", b);
    arr_u64("mt19937_seed99", c);
  }
  {  // std::shuffle of vector<long> (Word2Vec.cpp:367-373): pairwise (n <= 65535) and plain
    for (long n : {1L, 2L, 17L, 1000L, 70000L}) {
      std::mt19937 g(2024);
      std::vector<long> idx((size_t)n);
      std::iota(idx.begin(), idx.end(), 0);
      std::shuffle(idx.begin(), idx.end(), g);
      std::vector<uint64_t> v(idx.begin(), idx.end());
      char nm[64];
      std::snprintf(nm, sizeof nm, "shuffle_n%ld_seed2024", n);
      arr_u64(nm, v);
      std::vector<uint64_t> nxt{g()};
      std::snprintf(nm, sizeof nm, "shuffle_n%ld_seed2024_next_draw", n);
      arr_u64(nm, nxt);
    }
  }
  {  // unordered_map<size_t,uint8_t> iteration order (negative_sampling, :253-259)
    std::vector<std::vector<size_t>> seqs = {{5, 17, 3, 17, 99, 42}, {0, 13, 26, 1, 14}, {7, 7, 7, 7, 7, 7},
                                             {123456, 654321, 13, 26, 39, 5}};
    std::printf("\"nsmap_orders\": [");
    for (size_t s = 0; s < seqs.size(); ++s) {
      std::unordered_map<size_t, uint8_t> m;
      for (size_t k = 0; k + 1 < seqs[s].size(); ++k) m[seqs[s][k]] = 0;
      m[seqs[s].back()] = 1;
      std::printf("%s{\"inserts\": [", s ? "," : "");
      for (size_t k = 0; k < seqs[s].size(); ++k) std::printf("%s%zu", k ? "," : "", seqs[s][k]);
      std::printf("], \"order\": [");
      bool first = true;
      for (auto kv : m) { std::printf("%s[%zu,%d]", first ? "" : ",", kv.first, (int)kv.second); first = false; }
      std::printf("]}");
    }
    std::printf("],\n");
  }
  {  // build_vocab's unordered_map<string,int> order + std::sort (count desc) (:134-160)
    std::vector<std::string> toks;
    std::mt19937 g(3);
    std::uniform_int_distribution<int> z(0, 59);
    for (int i = 0; i < 3000; ++i) {
      int r = z(g);
      r = r * r / 60;  // skewed, many ties
      toks.push_back("w" + std::to_string(r));
    }
    std::unordered_map<std::string, int> cn;
    for (auto& w : toks) { if (cn.count(w) > 0) cn[w]++; else cn[w] = 1; }
    std::vector<std::pair<std::string, int>> kept;
    for (auto kv : cn) if (kv.second >= 5) kept.push_back(kv);
    std::vector<std::pair<std::string, int>*> ptrs;
    for (auto& k : kept) ptrs.push_back(&k);
    std::sort(ptrs.begin(), ptrs.end(), [](std::pair<std::string, int>* a, std::pair<std::string, int>* b) {
      return a->second > b->second;
    });
    std::printf("\"vocab_tokens_seed3\": [");
    for (size_t i = 0; i < toks.size(); ++i) std::printf("%s\"%s\"", i ? "," : "", toks[i].c_str());
    std::printf("],\n\"vocab_order_seed3\": [");
    for (size_t i = 0; i < ptrs.size(); ++i) std::printf("%s[\"%s\",%d]", i ? "," : "", ptrs[i]->first.c_str(), ptrs[i]->second);
    std::printf("],\n");
  }
  {  // Huffman over a count vector with ties (create_huffman_tree :32-79)
    std::vector<size_t> counts = {50, 30, 30, 20, 20, 20, 10, 10, 7, 5, 5, 5, 5, 3, 3, 2, 2, 2, 1, 1};
    std::vector<uint64_t> c, p, o;
    huffman_golden(counts, c, p, o);
    arr_u64("huffman_counts", std::vector<uint64_t>(counts.begin(), counts.end()));
    arr_u64("huffman_codes", c);
    arr_u64("huffman_points", p);
    arr_u64("huffman_offsets", o);
    std::vector<size_t> eq(33, 4);
    std::vector<uint64_t> c2, p2, o2;
    huffman_golden(eq, c2, p2, o2);
    arr_u64("huffman_eq33_codes", c2);
    arr_u64("huffman_eq33_points", p2);
    arr_u64("huffman_eq33_offsets", o2, true);
  }
  std::printf("}\n");
  return 0;
}
