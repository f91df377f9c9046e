// C bridge over the Word2Vec class (include/w2v_model.h).
#include <cstring>
#include <limits>
#include <sstream>
#include <stdexcept>
#include <string>

#include "Word2Vec.h"
#include "w2v_model.h"

struct w2v_model {
  Word2Vec w;
  std::string err;
  std::vector<int32_t> ids;       // w2v_model_file_samples
  std::vector<int64_t> offsets;
  w2v_model(int iter, int window, int min_count, int table_size, int dim, int negative, float sub, float a0,
            float a1, bool mean, int threads, const char* tm, const char* mdl)
      : w(iter, window, min_count, table_size, dim, negative, sub, a0, a1, mean, threads, tm, mdl) {}
};

namespace {

std::vector<std::vector<std::string>> parse(const char* text, int64_t len) {
  std::vector<std::vector<std::string>> out;
  std::istringstream lines(std::string(text, (size_t)len));
  std::string line;
  while (std::getline(lines, line)) {
    std::istringstream toks(line);
    std::vector<std::string> s;
    std::string t;
    while (toks >> t) s.push_back(t);
    out.push_back(std::move(s));
  }
  return out;
}

bool bad_word(w2v_model* m, int64_t i) {
  if (i >= 0 && i < (int64_t)m->w.vocab.size()) return false;
  m->err = "word index " + std::to_string(i) + " outside the vocab [0, " + std::to_string(m->w.vocab.size()) + ")";
  return true;
}

RMatrixXf* pick(w2v_model* m, int which) {
  return which == 0 ? &m->w.W : which == 1 ? &m->w.C : which == 2 ? &m->w.synapses1 : nullptr;
}

template <class F>
int guard(w2v_model* m, F f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    m->err = e.what();
  } catch (...) {
    m->err = "unknown error";
  }
  return 1;
}

}  // namespace

extern "C" {

w2v_model* w2v_model_new(int32_t iter, int32_t window, int32_t min_count, int32_t table_size, int32_t word_dim,
                         int32_t negative, float sub, float a0, float a1, int32_t cbow_mean, int32_t threads,
                         const char* tm, const char* mdl) {
  try {
    return new w2v_model(iter, window, min_count, table_size, word_dim, negative, sub, a0, a1, cbow_mean != 0,
                         threads, tm, mdl);
  } catch (...) {
    return nullptr;
  }
}
void w2v_model_free(w2v_model* m) { delete m; }
const char* w2v_model_last_error(w2v_model* m) { return m->err.c_str(); }
void w2v_model_seed(w2v_model* m, uint32_t s) { m->w.generator.seed(s); }
void w2v_model_options(w2v_model* m, int32_t gpu, int32_t replay, int32_t verbose) {
  m->w.gpu_device = gpu;
  m->w.replay_rng = replay != 0;
  m->w.verbose = verbose != 0;
}

void w2v_model_update_policy(w2v_model* m, int64_t hot_rows, int32_t private_rows, int32_t flush_centers,
                             float private_average, int64_t max_waves) {
  m->w.hot_rows = hot_rows;
  m->w.private_rows = private_rows;
  m->w.flush_centers = flush_centers;
  m->w.private_average = private_average;
  m->w.max_waves = max_waves;
}

void w2v_model_context_policy(w2v_model* m, int32_t context_rows, int32_t context_flush) {
  m->w.context_rows = context_rows;
  m->w.context_flush = context_flush;
}

void w2v_model_set_shared_negatives(w2v_model* m, int32_t on) { m->w.shared_negatives = on != 0; }

void w2v_model_replicas(w2v_model* m, const int32_t* devices, int32_t n, int64_t sync_words, int32_t overlap) {
  m->w.gpu_devices.assign(devices, devices + (n > 0 && devices ? n : 0));
  m->w.sync_words = sync_words;
  m->w.overlap_average = overlap != 0;
}

void w2v_model_replica_mode(w2v_model* m, int32_t mode) { m->w.replica_mode = mode; }

void w2v_model_set_gpu_ingest(w2v_model* m, int32_t on, int64_t chunk_bytes) {
  m->w.gpu_ingest = on != 0;
  m->w.ingest_chunk_bytes = chunk_bytes > 0 ? chunk_bytes : 0;
}

int w2v_model_build_vocab(w2v_model* m, const char* text, int64_t len) {
  return guard(m, [&] {
    auto s = parse(text, len);
    m->w.build_vocab(s);
  });
}
int w2v_model_train(w2v_model* m, const char* text, int64_t len) {
  return guard(m, [&] {
    auto s = parse(text, len);
    m->w.train(s);
  });
}
int w2v_model_train_ids(w2v_model* m, const int32_t* ids, const int64_t* off, int64_t n, int64_t tw) {
  return guard(m, [&] {
    std::vector<int32_t> i(ids, ids + off[n]);
    std::vector<int64_t> o(off, off + n + 1);
    m->w.train_ids(i, o, tw);
  });
}
int w2v_model_build_vocab_file(w2v_model* m, const char* path, const char* format, int32_t threads) {
  return guard(m, [&] { m->w.build_vocab_file(path, format, threads); });
}

int w2v_model_train_file(w2v_model* m, const char* path, const char* format, int32_t threads) {
  return guard(m, [&] { m->w.train_file(path, format, threads); });
}

int w2v_model_file_samples(w2v_model* m, const char* path, const char* format, int32_t threads, int64_t* n_tokens,
                           int64_t* n_sentences, int64_t* train_words) {
  return guard(m, [&] {
    int64_t tw = 0;
    m->w.file_samples(path, format, threads, m->ids, m->offsets, tw);
    if (n_tokens) *n_tokens = (int64_t)m->ids.size();
    if (n_sentences) *n_sentences = (int64_t)m->offsets.size() - 1;
    if (train_words) *train_words = tw;
  });
}

int w2v_model_copy_samples(w2v_model* m, int32_t* ids, int64_t* offsets) {
  return guard(m, [&] {
    if (ids && !m->ids.empty()) std::memcpy(ids, m->ids.data(), m->ids.size() * sizeof(int32_t));
    if (offsets) std::memcpy(offsets, m->offsets.data(), m->offsets.size() * sizeof(int64_t));
  });
}

int w2v_model_init_weights(w2v_model* m) {
  return guard(m, [&] { m->w.init_weights(m->w.vocab.size()); });
}

int64_t w2v_model_vocab_size(w2v_model* m) { return (int64_t)m->w.vocab.size(); }
// Out-of-range word indices: NULL / -1 / NaN / 1, with the message in last_error.
const char* w2v_model_word(w2v_model* m, int64_t i) {
  return bad_word(m, i) ? nullptr : m->w.vocab[(size_t)i]->text.c_str();
}
int64_t w2v_model_word_count(w2v_model* m, int64_t i) {
  return bad_word(m, i) ? -1 : (int64_t)m->w.vocab[(size_t)i]->count;
}
float w2v_model_sample_probability(w2v_model* m, int64_t i) {
  return bad_word(m, i) ? std::numeric_limits<float>::quiet_NaN() : m->w.vocab[(size_t)i]->sample_probability;
}
int64_t w2v_model_path_length(w2v_model* m, int64_t i) {
  return bad_word(m, i) ? -1 : (int64_t)m->w.vocab[(size_t)i]->codes.size();
}
int w2v_model_path(w2v_model* m, int64_t i, uint8_t* codes, int32_t* points) {
  if (bad_word(m, i)) return 1;
  const Word* w = m->w.vocab[(size_t)i];
  for (size_t k = 0; k < w->codes.size(); ++k) {
    codes[k] = (uint8_t)w->codes[k];
    points[k] = (int32_t)w->points[k];
  }
  return 0;
}
int64_t w2v_model_table_length(w2v_model* m) { return (int64_t)m->w.table.size(); }
int w2v_model_table(w2v_model* m, uint32_t* out) {
  for (size_t k = 0; k < m->w.table.size(); ++k) out[k] = (uint32_t)m->w.table[k];
  return 0;
}

int64_t w2v_model_rows(w2v_model* m, int32_t which) {
  RMatrixXf* M = pick(m, which);
  return M ? (int64_t)M->rows() : -1;
}
int w2v_model_get_matrix(w2v_model* m, int32_t which, float* out) {
  RMatrixXf* M = pick(m, which);
  if (!M) return 1;
  std::memcpy(out, M->data(), sizeof(float) * (size_t)M->size());
  return 0;
}
int w2v_model_set_matrix(w2v_model* m, int32_t which, const float* in, int64_t rows, int64_t cols) {
  RMatrixXf* M = pick(m, which);
  if (!M) {
    m->err = "bad matrix selector";
    return 1;
  }
  if (rows < 0 || cols != m->w.word_dim || (rows > 0 && !in)) {
    m->err = "set_matrix: expected rows >= 0 x word_dim (" + std::to_string(m->w.word_dim) + ") columns, got " +
             std::to_string(rows) + " x " + std::to_string(cols);
    return 1;
  }
  M->resize((RMatrixXf::Index)rows, m->w.word_dim);
  std::memcpy(M->data(), in, sizeof(float) * (size_t)M->size());
  return 0;
}

int w2v_model_train_sentence(w2v_model* m, const int32_t* ids, int64_t n, float alpha, int32_t cbow) {
  return guard(m, [&] {
    std::vector<Word*> s;
    for (int64_t k = 0; k < n; ++k) {
      if (ids[k] < 0 || (size_t)ids[k] >= m->w.vocab.size()) throw std::out_of_range("train_sentence: token id out of vocab");
      s.push_back(m->w.vocab[(size_t)ids[k]]);
    }
    if (cbow) m->w.train_sentence_cbow(s, alpha);
    else m->w.train_sentence_sg(s, alpha);
  });
}
int w2v_model_negative_sampling(w2v_model* m, int64_t word, float* x, float* grad, int32_t which, float alpha) {
  if (bad_word(m, word)) return 1;
  return guard(m, [&] {
    RowVectorXf xv((w2v_dense::Index)m->w.word_dim), gv((w2v_dense::Index)m->w.word_dim);
    std::memcpy(xv.data(), x, sizeof(float) * (size_t)m->w.word_dim);
    std::memcpy(gv.data(), grad, sizeof(float) * (size_t)m->w.word_dim);
    m->w.negative_sampling(m->w.vocab[(size_t)word], xv, gv, which == 0 ? m->w.W : m->w.C, alpha);
    std::memcpy(grad, gv.data(), sizeof(float) * (size_t)m->w.word_dim);
  });
}
int w2v_model_hierarchical_softmax(w2v_model* m, int64_t word, float* x, float* grad, float alpha) {
  if (bad_word(m, word)) return 1;
  return guard(m, [&] {
    RowVectorXf xv((w2v_dense::Index)m->w.word_dim), gv((w2v_dense::Index)m->w.word_dim);
    std::memcpy(xv.data(), x, sizeof(float) * (size_t)m->w.word_dim);
    std::memcpy(gv.data(), grad, sizeof(float) * (size_t)m->w.word_dim);
    m->w.hierarchical_softmax(m->w.vocab[(size_t)word], xv, gv, alpha);
    std::memcpy(grad, gv.data(), sizeof(float) * (size_t)m->w.word_dim);
  });
}

int w2v_model_save(w2v_model* m, const char* path, int32_t which, int32_t binary) {
  return guard(m, [&] {
    RMatrixXf* M = pick(m, which);
    if (!M) throw std::runtime_error("bad matrix selector");
    m->w.save_word2vec(path, *M, binary != 0);
  });
}
int w2v_model_load(w2v_model* m, const char* path, int32_t binary) {
  return guard(m, [&] { m->w.load_word2vec(path, binary != 0); });
}
int w2v_model_save_checkpoint(w2v_model* m, const char* path) {
  return guard(m, [&] { m->w.save_checkpoint(path); });
}
int w2v_model_load_checkpoint(w2v_model* m, const char* path) {
  return guard(m, [&] { m->w.load_checkpoint(path); });
}
int64_t w2v_model_current_words(w2v_model* m) { return m->w.current_words(); }
int64_t w2v_model_replica_rounds(w2v_model* m) { return m->w.replica_rounds; }
double w2v_model_replica_max_diff(w2v_model* m) { return m->w.replica_max_diff; }
int w2v_model_set_checkpoint_path(w2v_model* m, const char* path) {
  return guard(m, [&] { m->w.checkpoint_path = path ? path : ""; });
}
int64_t w2v_model_epochs_done(w2v_model* m) { return m->w.epochs_done(); }
double w2v_model_epoch_seconds(w2v_model* m, int64_t i) {
  return (i >= 0 && i < (int64_t)m->w.epoch_seconds.size()) ? m->w.epoch_seconds[(size_t)i] : -1.0;
}
int w2v_model_save_vocab(w2v_model* m, const char* path) {
  return guard(m, [&] { m->w.save_vocab(path); });
}
int w2v_model_read_vocab(w2v_model* m, const char* path) {
  return guard(m, [&] { m->w.read_vocab(path); });
}

// The reference's public vocabulary products (Word2Vec.h:70-72), e.g. after
// read_vocab, which builds none of them (Word2Vec.cpp:171-196).
int w2v_model_create_huffman_tree(w2v_model* m) {
  return guard(m, [&] { m->w.create_huffman_tree(); });
}
int w2v_model_make_table(w2v_model* m) {
  return guard(m, [&] { m->w.make_table(); });
}
int w2v_model_precalc_sampling(w2v_model* m) {
  return guard(m, [&] { m->w.precalc_sampling(); });
}

}  // extern "C"
