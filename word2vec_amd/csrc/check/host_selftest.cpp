// host_selftest.cpp — exercises the host side of the boundary (the Word2Vec
// class's vocabulary, Huffman, table, sampling, weight init, corpus readers,
// vector/vocab files, and the C bridge's argument checks) with no device call,
// for the AddressSanitizer / UndefinedBehaviorSanitizer build
// (make -C word2vec_amd/csrc asan; tests/test_host_sanitizers.py).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "Word2Vec.h"
#include "w2v_host.h"
#include "w2v_model.h"

namespace {

int failures = 0;
void expect(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    ++failures;
  }
}

std::vector<std::vector<std::string>> corpus(int n_sent, int len, int vmax, unsigned seed) {
  std::mt19937 g(seed);
  std::vector<std::vector<std::string>> out;
  for (int s = 0; s < n_sent; ++s) {
    std::vector<std::string> sent;
    for (int t = 0; t < len; ++t) {
      // Zipf-ish: rank = floor(vmax^u) - 1
      const double u = std::uniform_real_distribution<double>(0.0, 1.0)(g);
      sent.push_back("w" + std::to_string((int)std::pow((double)vmax, u) - 1));
    }
    out.push_back(sent);
  }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  auto sents = corpus(60, 120, 400, 7);
  for (const char* method : {"hs", "ns"}) {
    for (const char* model : {"sg", "cbow"}) {
      const bool ns = std::string(method) == "ns";
      Word2Vec w(1, 5, 2, 20000, 24, ns ? 5 : 0, 1e-3f, 0.025f, 1e-6f, true, 1, method, model);
      w.generator.seed(11);
      w.build_vocab(sents);
      expect(!w.vocab.empty(), "vocab built");
      for (size_t i = 1; i < w.vocab.size(); ++i) expect(w.vocab[i - 1]->count >= w.vocab[i]->count, "sorted by count");
      if (!ns) {
        for (Word* v : w.vocab) expect(v->codes.size() == v->points.size() && !v->codes.empty(), "huffman path");
      } else {
        expect(w.table.size() == 20000, "table size");
      }
      w.init_weights(w.vocab.size());
      expect(w.W.rows() == (long)w.vocab.size(), "W rows");
      auto samples = w.build_sample(sents);
      expect(samples.size() == sents.size(), "build_sample");
      const std::string vec = dir + "/selftest_vec.txt", vecb = dir + "/selftest_vec.bin", voc = dir + "/selftest_vocab.txt";
      w.save_word2vec(vec, w.W, false);
      w.save_word2vec(vecb, w.W, true);
      w.save_vocab(voc);
      RMatrixXf keep = w.W;
      w.load_word2vec(vecb, true);
      bool same = true;
      for (long k = 0; k < keep.size(); ++k) same = same && keep.data()[k] == w.W.data()[k];
      expect(same, "binary round trip");
      w.load_word2vec(vec, false);
      Word2Vec r;
      r.read_vocab(voc);
      expect(r.vocab.size() == w.vocab.size(), "read_vocab");
    }
  }
  {  // corpus file readers
    const std::string path = dir + "/selftest_corpus.txt";
    {
      std::ofstream f(path);
      for (auto& s : sents) {
        for (size_t t = 0; t < s.size(); ++t) f << (t ? " " : "") << s[t];
        f << "\n";
      }
    }
    Word2Vec a(1, 5, 2, 20000, 16, 5, 1e-3f, 0.025f, 1e-6f, true, 1, "ns", "sg");
    Word2Vec b(1, 5, 2, 20000, 16, 5, 1e-3f, 0.025f, 1e-6f, true, 1, "ns", "sg");
    a.build_vocab(sents);
    b.build_vocab_file(path, "lines", 2);
    expect(a.vocab.size() == b.vocab.size(), "build_vocab_file == build_vocab");
    for (size_t i = 0; i < a.vocab.size() && i < b.vocab.size(); ++i)
      expect(a.vocab[i]->text == b.vocab[i]->text && a.vocab[i]->count == b.vocab[i]->count, "same vocab order");
    std::vector<int32_t> ids;
    std::vector<int64_t> off;
    int64_t tw = 0;
    b.file_samples(path, "text8", 3, ids, off, tw);
    expect(tw == 60 * 120, "train_words");
  }
  {  // C bridge argument checks
    w2v_model* m = w2v_model_new(1, 5, 2, 20000, 16, 5, 1e-3f, 0.025f, 1e-6f, 1, 1, "ns", "sg");
    std::string text;
    for (auto& s : sents) {
      for (auto& t : s) text += t + " ";
      text += "\n";
    }
    expect(w2v_model_build_vocab(m, text.data(), (int64_t)text.size()) == 0, "bridge build_vocab");
    expect(w2v_model_word(m, -1) == nullptr, "word(-1) rejected");
    expect(w2v_model_word(m, 1 << 30) == nullptr, "word(big) rejected");
    expect(w2v_model_word_count(m, 1 << 30) == -1, "count(big) rejected");
    std::vector<float> mat(4 * 16, 0.5f);
    expect(w2v_model_set_matrix(m, 0, mat.data(), 4, 17) != 0, "set_matrix wrong width rejected");
    expect(w2v_model_set_matrix(m, 0, mat.data(), 4, 16) == 0, "set_matrix ok");
    int32_t bad[2] = {0, 1 << 30};
    expect(w2v_model_train_sentence(m, bad, 2, 0.01f, 0) != 0, "train_sentence bad id rejected");
    float x[16] = {0}, g[16] = {0};
    expect(w2v_model_negative_sampling(m, 1 << 30, x, g, 1, 0.01f) != 0, "negative_sampling bad id rejected");
    w2v_model_free(m);
  }
  std::printf("host selftest: %d failure(s)\n", failures);
  return failures ? 1 : 0;
}
