// Word2Vec.cpp — host side of the Word2Vec class API (include/Word2Vec.h).
//
// Each method keeps the reference's contract (/root/reference/Word2Vec.cpp,
// cited per method); the vocabulary products are computed by the bit-exact
// restatements in vocab_products.cpp, and every model update runs on the GPU
// through include/w2v_dev.h.
#include "Word2Vec.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <numeric>
#include <set>
#include <sstream>
#include <stdexcept>

#include "w2v_corpus.h"
#include "w2v_dev.h"
#include "w2v_host.h"

namespace {

bool count_desc(Word* a, Word* b) { return a->count > b->count; }  // Word2Vec.cpp:3-6

}  // namespace

Word2Vec::~Word2Vec(void) {
  if (dev_) w2v_dev_destroy(dev_);
}

// Word2Vec.cpp:12-17. cbow_mean is initialised from the argument here (the
// reference leaves it uninitialised: its initialiser list omits it).
Word2Vec::Word2Vec(int iter_, int window_, int min_count_, int table_size_, int word_dim_, int negative_,
                   float subsample_threshold_, float init_alpha_, float min_alpha_, bool cbow_mean_,
                   int num_threads_, std::string train_method_, std::string model_)
    : iter(iter_), window(window_), min_count(min_count_), table_size(table_size_), word_dim(word_dim_),
      negative(negative_), subsample_threshold(subsample_threshold_), init_alpha(init_alpha_),
      min_alpha(min_alpha_), num_threads(num_threads_), cbow_mean(cbow_mean_), phrase(false),
      train_method(train_method_), model(model_), generator(rd()),
      distribution_window(0, window_ < 1 ? 0 : window_ - 1), distribution_table(0, table_size_ - 1),
      uni_dis(0.0, 1.0) {}

// Word2Vec.cpp:19-30: one sentence per line, whitespace-separated tokens.
std::vector<std::vector<std::string>> Word2Vec::line_docs(std::string filename) {
  std::vector<std::vector<std::string>> out;
  std::ifstream in(filename);
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream toks(line);
    out.emplace_back(std::istream_iterator<std::string>{toks}, std::istream_iterator<std::string>{});
  }
  return out;
}

// Declared but never defined by the reference (Word2Vec.h:69); kept as a no-op.
void Word2Vec::reduce_vocab() {}

// Word2Vec.cpp:32-79 (codes/points only: the reference's internal nodes are
// unreachable from the public members).
void Word2Vec::create_huffman_tree() {
  dev_vocab_stale_ = true;
  const int64_t V = (int64_t)vocab.size();
  if (V < 2) return;
  std::vector<int64_t> counts((size_t)V);
  for (int64_t i = 0; i < V; ++i) counts[(size_t)i] = (int64_t)vocab[(size_t)i]->count;
  std::vector<int64_t> off((size_t)V + 1);
  const int64_t total = w2v_host_huffman(counts.data(), V, nullptr, nullptr, off.data(), 0);
  std::vector<uint8_t> codes((size_t)std::max<int64_t>(total, 1));
  std::vector<int32_t> points((size_t)std::max<int64_t>(total, 1));
  w2v_host_huffman(counts.data(), V, codes.data(), points.data(), off.data(), total);
  for (int64_t w = 0; w < V; ++w) {
    Word* word = vocab[(size_t)w];
    word->codes.assign(codes.begin() + off[(size_t)w], codes.begin() + off[(size_t)w + 1]);
    word->points.assign(points.begin() + off[(size_t)w], points.begin() + off[(size_t)w + 1]);
  }
}

// Word2Vec.cpp:81-113 (same table, built from its V+1 boundaries).
void Word2Vec::make_table() {
  dev_vocab_stale_ = true;
  const int64_t V = (int64_t)vocab.size();
  table.assign((size_t)table_size, 0);
  if (V == 0) return;
  std::vector<int64_t> counts((size_t)V), b((size_t)V + 1);
  for (int64_t i = 0; i < V; ++i) counts[(size_t)i] = (int64_t)vocab[(size_t)i]->count;
  w2v_host_table_bounds(counts.data(), V, table_size, b.data());
  for (int64_t w = 0; w < V; ++w)
    std::fill(table.begin() + b[(size_t)w], table.begin() + b[(size_t)w + 1], (size_t)w);
}

// Word2Vec.cpp:115-130.
void Word2Vec::precalc_sampling() {
  dev_vocab_stale_ = true;
  const int64_t V = (int64_t)vocab.size();
  std::vector<int64_t> counts((size_t)V);
  std::vector<float> p((size_t)V);
  for (int64_t i = 0; i < V; ++i) counts[(size_t)i] = (int64_t)vocab[(size_t)i]->count;
  w2v_host_sample_probs(counts.data(), V, subsample_threshold, p.data());
  for (int64_t i = 0; i < V; ++i) vocab[(size_t)i]->sample_probability = p[(size_t)i];
}

// Word2Vec.cpp:132-169: count in corpus order with unordered_map<string,int>,
// keep >= min_count in the map's iteration order, std::sort by count desc.
void Word2Vec::build_vocab(std::vector<std::vector<std::string>>& sentences) {
  std::unordered_map<std::string, int> tally;
  for (auto& sentence : sentences)
    for (auto& w : sentence) {
      if (tally.count(w) > 0) tally[w]++;
      else tally[w] = 1;
    }
  finish_vocab(tally);
}

// The counting map's iteration order depends only on the order in which the
// distinct words were first inserted, so a file's counts inserted in order of
// first occurrence give the map build_vocab builds (corpus.cpp).
void Word2Vec::build_vocab_file(const std::string& path, const std::string& format, int threads) {
  const w2v_corpus::File f(path);
  const w2v_corpus::Counts c = w2v_corpus::count_words(f, w2v_corpus::parse_format(format), threads);
  std::unordered_map<std::string, int> tally;
  for (const auto& wc : c.words) tally[wc.first] = (int)wc.second;
  finish_vocab(tally);
}

void Word2Vec::file_samples(const std::string& path, const std::string& format, int threads,
                            std::vector<int32_t>& ids, std::vector<int64_t>& offsets, int64_t& train_words) {
  std::unordered_map<std::string, int32_t> index;
  index.reserve(vocab.size());
  for (const Word* w : vocab) index[w->text] = (int32_t)w->index;
  const w2v_corpus::File f(path);
  w2v_corpus::Samples s = w2v_corpus::samples(f, w2v_corpus::parse_format(format), threads, index);
  ids.swap(s.ids);
  offsets.swap(s.offsets);
  train_words = s.raw_tokens;
}

void Word2Vec::train_file(const std::string& path, const std::string& format, int threads) {
  std::vector<int32_t> ids;
  std::vector<int64_t> offsets;
  int64_t train_words = 0;
  file_samples(path, format, threads, ids, offsets, train_words);
  train_ids(ids, offsets, train_words);
}

// Word2Vec.cpp:143-168: keep >= min_count in the map's iteration order,
// std::sort by count desc, index, then the vocab products.
void Word2Vec::finish_vocab(std::unordered_map<std::string, int>& tally) {
  for (auto kv : tally) {
    if (kv.second < min_count) continue;
    Word* w = new Word(0, (size_t)kv.second, kv.first);
    vocab.push_back(w);
    vocab_hash[w->text] = WordP(w);
  }
  std::sort(vocab.begin(), vocab.end(), count_desc);
  for (size_t i = 0; i < vocab.size(); ++i) {
    vocab[i]->index = i;
    idx2word.push_back(vocab[i]->text);
  }
  if (train_method == "hs") create_huffman_tree();
  if (negative) make_table();
  precalc_sampling();
}

// Word2Vec.cpp:171-177.
void Word2Vec::save_vocab(std::string vocab_filename) {
  std::ofstream out(vocab_filename, std::ofstream::out);
  for (auto& v : vocab) out << v->index << " " << v->count << " " << v->text << std::endl;
}

// Word2Vec.cpp:179-196.
void Word2Vec::read_vocab(std::string vocab_filename) {
  dev_vocab_stale_ = true;
  std::ifstream in(vocab_filename);
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream iss(line);
    size_t index, count;
    std::string text;
    iss >> index >> count >> text;
    Word* w = new Word(index, count, text);
    vocab.push_back(w);
    vocab_hash[w->text] = WordP(w);
  }
}

bool Word2Vec::uses_C() const { return negative > 0 || model == "cbow"; }

// Word2Vec.cpp:198-210: W = U(-0.5, 0.5) / dim drawn row-major from the
// shared generator. synapses1 = 0 for hs; C = 0 when negative sampling uses
// it. For cbow + hs, C (the CBOW input matrix) is drawn like W right after it:
// the reference reads an unallocated C there (documented deviation).
void Word2Vec::init_weights(size_t vocab_size) {
  std::uniform_real_distribution<float> dist(-0.5, 0.5);
  const size_t d = (size_t)word_dim;
  W.resize((w2v_dense::Index)vocab_size, (w2v_dense::Index)d);
  float* w = W.data();
  for (size_t k = 0; k < vocab_size * d; ++k) w[k] = dist(generator);
  for (size_t k = 0; k < vocab_size * d; ++k) w[k] = w[k] / (float)word_dim;
  synapses1 = RMatrixXf();
  C = RMatrixXf();
  if (train_method == "hs") synapses1 = RMatrixXf::Zero((w2v_dense::Index)(vocab_size ? vocab_size - 1 : 0), d);
  if (model == "cbow" && train_method == "hs") {
    C.resize((w2v_dense::Index)vocab_size, (w2v_dense::Index)d);
    float* c = C.data();
    for (size_t k = 0; k < vocab_size * d; ++k) c[k] = dist(generator);
    for (size_t k = 0; k < vocab_size * d; ++k) c[k] = c[k] / (float)word_dim;
  } else if (uses_C()) {
    C = RMatrixXf::Zero((w2v_dense::Index)vocab_size, d);
  }
}

// Word2Vec.cpp:212-230.
std::vector<std::vector<Word*>> Word2Vec::build_sample(std::vector<std::vector<std::string>>& data) {
  std::vector<std::vector<Word*>> samples;
  samples.reserve(data.size());
  for (auto& sentence : data) {
    std::vector<Word*> kept;
    for (auto& text : sentence) {
      auto it = vocab_hash.find(text);
      if (it != vocab_hash.end()) kept.push_back(it->second.get());
    }
    samples.push_back(std::move(kept));
  }
  return samples;
}

// ---------------------------------------------------------------------------
// Device plumbing
// ---------------------------------------------------------------------------
void Word2Vec::check(int rc, const char* what) {
  if (rc == W2V_OK) return;
  last_error = std::string(what) + ": " + w2v_dev_last_error();
  throw std::runtime_error("word2vec_amd: " + last_error);
}

void Word2Vec::ensure_device() {
  w2v_dev_config cfg;
  std::memset(&cfg, 0, sizeof(cfg));
  cfg.word_dim = word_dim;
  cfg.window = window;
  cfg.negative = negative;
  cfg.hs = train_method == "hs" ? 1 : 0;
  cfg.cbow = model == "cbow" ? 1 : 0;
  cfg.cbow_mean = cbow_mean ? 1 : 0;
  cfg.iter = iter;
  cfg.init_alpha = init_alpha;
  cfg.min_alpha = min_alpha;
  cfg.table_size = table_size;
  cfg.device = gpu_device;
  if (dev_ && std::memcmp(&cfg, &dev_cfg_, sizeof(cfg)) == 0) return;
  if (dev_) w2v_dev_destroy(dev_);
  dev_ = nullptr;
  dev_vocab_stale_ = true;
  check(w2v_dev_create(&cfg, &dev_), "w2v_dev_create");
  dev_cfg_ = cfg;
}

void Word2Vec::upload_vocab_products() {
  if (!dev_vocab_stale_) return;
  const int64_t V = (int64_t)vocab.size();
  std::vector<float> keep((size_t)V);
  std::vector<int64_t> counts((size_t)V);
  for (int64_t i = 0; i < V; ++i) {
    keep[(size_t)i] = vocab[(size_t)i]->sample_probability;
    counts[(size_t)i] = (int64_t)vocab[(size_t)i]->count;
  }
  std::vector<int64_t> bounds;
  if (negative > 0) {
    bounds.resize((size_t)V + 1);
    w2v_host_table_bounds(counts.data(), V, table_size, bounds.data());
  }
  std::vector<uint8_t> codes;
  std::vector<int32_t> points;
  std::vector<int64_t> off;
  if (train_method == "hs") {
    off.assign((size_t)V + 1, 0);
    for (int64_t w = 0; w < V; ++w) {
      const Word* word = vocab[(size_t)w];
      for (size_t k = 0; k < word->codes.size(); ++k) {
        codes.push_back((uint8_t)word->codes[k]);
        points.push_back((int32_t)word->points[k]);
      }
      off[(size_t)w + 1] = (int64_t)codes.size();
    }
    if (codes.empty()) { codes.push_back(0); points.push_back(0); }
  }
  check(w2v_dev_upload_vocab(dev_, V, keep.data(), bounds.empty() ? nullptr : bounds.data(),
                             codes.empty() ? nullptr : codes.data(), points.empty() ? nullptr : points.data(),
                             off.empty() ? nullptr : off.data()),
        "w2v_dev_upload_vocab");
  dev_vocab_stale_ = false;
}

// The draws the reference makes for one pass over `order`, in its order
// (Word2Vec.cpp:279-310 CBOW, :325-349 SG, :254-255 NS), taken from this
// object's generator, with each sentence's start recorded.
void Word2Vec::append_reference_draws(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets,
                                      const std::vector<long>& order, std::vector<uint32_t>& stream,
                                      std::vector<int64_t>& stream_off, int64_t epoch) {
  const int64_t n = (int64_t)offsets.size() - 1;
  const bool cbow = model == "cbow";
  for (long s : order) {
    stream_off[(size_t)(epoch * n + s)] = (int64_t)stream.size();
    const int32_t* sent = ids.data() + offsets[(size_t)s];
    const int len = (int)(offsets[(size_t)s + 1] - offsets[(size_t)s]);
    for (int i = 0; i < len; ++i) {
      const float u = uni_dis(generator);
      uint32_t bits;
      std::memcpy(&bits, &u, 4);
      stream.push_back(bits);
      if (vocab[(size_t)sent[i]]->sample_probability < u) continue;
      const int rw = distribution_window(generator);
      stream.push_back((uint32_t)rw);
      const int lo = std::max(0, i - window + rw), hi = std::min(len, i + window + 1 - rw);
      if (cbow) {
        if (hi - lo - 1 <= 0) continue;
        for (int k = 0; k < negative; ++k) stream.push_back((uint32_t)distribution_table(generator));
      } else {
        for (int j = lo; j < hi; ++j) {
          if (j == i) continue;
          for (int k = 0; k < negative; ++k) stream.push_back((uint32_t)distribution_table(generator));
        }
      }
    }
  }
}

// The epoch loop of Word2Vec.cpp:367-395 with the model resident in HBM.
void Word2Vec::run_epochs(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets,
                          int64_t train_words) {
  ensure_device();
  upload_vocab_products();
  check(w2v_dev_upload_model(dev_, W.data(), uses_C() ? C.data() : nullptr,
                             train_method == "hs" ? synapses1.data() : nullptr),
        "w2v_dev_upload_model");
  const int64_t n = (int64_t)offsets.size() - 1;
  check(w2v_dev_upload_corpus(dev_, ids.data(), (int64_t)ids.size(), offsets.data(), n, train_words),
        "w2v_dev_upload_corpus");
  check(w2v_dev_set_fixed_alpha(dev_, 0.0f), "w2v_dev_set_fixed_alpha");
  check(w2v_dev_set_hot_rows(dev_, hot_rows), "w2v_dev_set_hot_rows");
  check(w2v_dev_set_private_rows(dev_, private_rows), "w2v_dev_set_private_rows");
  check(w2v_dev_set_private_sync(dev_, flush_centers, private_average), "w2v_dev_set_private_sync");
  check(w2v_dev_set_max_waves(dev_, max_waves), "w2v_dev_set_max_waves");
  check(w2v_dev_set_context_private(dev_, context_rows, context_flush), "w2v_dev_set_context_private");
  check(w2v_dev_set_update(dev_, shared_negatives ? W2V_UPDATE_SHARED_NEGATIVES : W2V_UPDATE_PER_PAIR),
        "w2v_dev_set_update");
  check(w2v_dev_set_progress(dev_, 0), "w2v_dev_set_progress");  // current_words = 0 (:359)
  std::vector<long> sample_idx((size_t)n);
  std::iota(sample_idx.begin(), sample_idx.end(), 0);
  std::vector<std::vector<int64_t>> orders;
  if (replay_rng) {
    std::vector<uint32_t> stream;
    std::vector<int64_t> stream_off((size_t)(n * iter), 0);
    for (int it = 0; it < iter; ++it) {
      std::shuffle(sample_idx.begin(), sample_idx.end(), generator);
      orders.emplace_back(sample_idx.begin(), sample_idx.end());
      append_reference_draws(ids, offsets, sample_idx, stream, stream_off, it);
    }
    check(w2v_dev_upload_replay(dev_, stream.data(), (int64_t)stream.size(), stream_off.data(),
                                (int64_t)stream_off.size()),
          "w2v_dev_upload_replay");
    check(w2v_dev_set_rng(dev_, W2V_RNG_REPLAY, 0), "w2v_dev_set_rng");
    check(w2v_dev_set_schedule(dev_, W2V_SCHED_SEQUENTIAL), "w2v_dev_set_schedule");
  } else {
    const uint64_t key = ((uint64_t)generator() << 32) | (uint64_t)generator();
    check(w2v_dev_set_rng(dev_, W2V_RNG_PHILOX, key), "w2v_dev_set_rng");
    check(w2v_dev_set_schedule(dev_, W2V_SCHED_PARALLEL), "w2v_dev_set_schedule");
  }
  for (int it = 0; it < iter; ++it) {
    if (!replay_rng) {
      std::shuffle(sample_idx.begin(), sample_idx.end(), generator);
      orders.emplace_back(sample_idx.begin(), sample_idx.end());
    }
    w2v_dev_stats st;
    std::memset(&st, 0, sizeof(st));
    check(w2v_dev_train_epoch(dev_, it, orders[(size_t)it].data(), &st), "w2v_dev_train_epoch");
    int64_t cw = 0;
    check(w2v_dev_get_progress(dev_, &cw), "w2v_dev_get_progress");
    if (verbose) {
      std::printf("\rinit_alpha: %f  Progress: %f%% ", init_alpha, 100.0 / iter * cw / train_words);
      std::fflush(stdout);
    }
  }
  int64_t cw = 0;
  check(w2v_dev_get_progress(dev_, &cw), "w2v_dev_get_progress");
  cur_words_ = cw;
  check(w2v_dev_download_model(dev_, W.data(), uses_C() ? C.data() : nullptr,
                               train_method == "hs" ? synapses1.data() : nullptr),
        "w2v_dev_download_model");
  if (verbose) std::printf("\n");
}

// Word2Vec.cpp:356-396.
void Word2Vec::train(std::vector<std::vector<std::string>>& sentences) {
  init_weights(vocab.size());
  int64_t train_words = 0;
  for (auto& s : sentences) train_words += (int64_t)s.size();
  std::vector<int32_t> ids;
  std::vector<int64_t> offsets(1, 0);
  for (auto& sentence : sentences) {  // build_sample as token ids
    for (auto& text : sentence) {
      auto it = vocab_hash.find(text);
      if (it != vocab_hash.end()) ids.push_back((int32_t)it->second->index);
    }
    offsets.push_back((int64_t)ids.size());
  }
  run_epochs(ids, offsets, train_words);
}

void Word2Vec::train_ids(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets,
                         int64_t train_words) {
  init_weights(vocab.size());
  run_epochs(ids, offsets, train_words);
}

// ---------------------------------------------------------------------------
// Per-call hot-path methods: same contract, arithmetic on the device.
// ---------------------------------------------------------------------------
void Word2Vec::apply_rows(RMatrixXf& M, int, const std::vector<size_t>& rows, const std::vector<uint8_t>& codes,
                          RowVectorXf& x, RowVectorXf& grad, float alpha, bool hs_form) {
  ensure_device();
  const size_t d = (size_t)word_dim, n = rows.size();
  std::vector<float> buf(n * d);
  for (size_t t = 0; t < n; ++t) std::memcpy(&buf[t * d], M.row((w2v_dense::Index)rows[t]).data(), d * 4);
  check(w2v_dev_apply_rows(dev_, buf.data(), codes.data(), (int32_t)n, x.data(), grad.data(), alpha,
                           hs_form ? 1 : 0),
        "w2v_dev_apply_rows");
  for (size_t t = 0; t < n; ++t) std::memcpy(M.row((w2v_dense::Index)rows[t]).data(), &buf[t * d], d * 4);
}

// Word2Vec.cpp:232-249.
RowVectorXf& Word2Vec::hierarchical_softmax(Word* predict_word, RowVectorXf& project_rep,
                                            RowVectorXf& project_grad, float alpha) {
  std::vector<size_t> rows(predict_word->points.begin(), predict_word->points.end());
  std::vector<uint8_t> codes(predict_word->codes.begin(), predict_word->codes.end());
  if (!rows.empty()) apply_rows(synapses1, 2, rows, codes, project_rep, project_grad, alpha, true);
  return project_grad;
}

// Word2Vec.cpp:251-271: the same target map (negatives from the shared
// generator, the positive set last), visited in the map's order.
RowVectorXf& Word2Vec::negative_sampling(Word* predict_word, RowVectorXf& project_rep, RowVectorXf& project_grad,
                                         RMatrixXf& target_matrix, float alpha) {
  std::unordered_map<size_t, uint8_t> targets;
  for (int i = 0; i < negative; ++i) targets[table[(size_t)distribution_table(generator)]] = 0;
  targets[predict_word->index] = 1;
  std::vector<size_t> rows;
  std::vector<uint8_t> codes;
  for (auto kv : targets) {
    rows.push_back(kv.first);
    codes.push_back((uint8_t)(1 - kv.second));
  }
  apply_rows(target_matrix, &target_matrix == &W ? 0 : 1, rows, codes, project_rep, project_grad, alpha, false);
  return project_grad;
}

// Word2Vec.cpp:273-317 and :319-353 on one sentence: the reference's draws for
// it come from this object's generator (same order), the update runs on the
// device with the caller's alpha.
void Word2Vec::train_one_sentence(std::vector<Word*>& sentence, float alpha, bool cbow) {
  const std::string saved = model;
  model = cbow ? "cbow" : "sg";
  try {
    std::vector<int32_t> ids;
    for (Word* w : sentence) ids.push_back((int32_t)w->index);
    std::vector<int64_t> off{0, (int64_t)ids.size()};
    ensure_device();
    upload_vocab_products();
    check(w2v_dev_upload_model(dev_, W.data(), uses_C() && C.size() ? C.data() : nullptr,
                               train_method == "hs" ? synapses1.data() : nullptr),
          "w2v_dev_upload_model");
    check(w2v_dev_upload_corpus(dev_, ids.data(), (int64_t)ids.size(), off.data(), 1,
                                std::max<int64_t>(1, (int64_t)ids.size())),
          "w2v_dev_upload_corpus");
    std::vector<uint32_t> stream;
    std::vector<int64_t> soff(1, 0);
    append_reference_draws(ids, off, std::vector<long>{0}, stream, soff, 0);
    check(w2v_dev_upload_replay(dev_, stream.data(), (int64_t)stream.size(), soff.data(), 1),
          "w2v_dev_upload_replay");
    check(w2v_dev_set_rng(dev_, W2V_RNG_REPLAY, 0), "w2v_dev_set_rng");
    check(w2v_dev_set_schedule(dev_, W2V_SCHED_SEQUENTIAL), "w2v_dev_set_schedule");
    check(w2v_dev_set_fixed_alpha(dev_, alpha), "w2v_dev_set_fixed_alpha");
    check(w2v_dev_train_epoch(dev_, 0, nullptr, nullptr), "w2v_dev_train_epoch");
    check(w2v_dev_set_fixed_alpha(dev_, 0.0f), "w2v_dev_set_fixed_alpha");
    check(w2v_dev_download_model(dev_, W.data(), uses_C() && C.size() ? C.data() : nullptr,
                                 train_method == "hs" ? synapses1.data() : nullptr),
          "w2v_dev_download_model");
  } catch (...) {
    model = saved;
    throw;
  }
  model = saved;
}

void Word2Vec::train_sentence_cbow(std::vector<Word*>& sentence, float alpha) {
  train_one_sentence(sentence, alpha, true);
}

void Word2Vec::train_sentence_sg(std::vector<Word*>& sentence, float alpha) {
  train_one_sentence(sentence, alpha, false);
}

// ---------------------------------------------------------------------------
// Vector files (Word2Vec.cpp:398-495), same bytes.
// ---------------------------------------------------------------------------
void Word2Vec::save_word2vec(std::string filename, const RMatrixXf& data, bool binary) {
  IOFormat fmt(w2v_dense::StreamPrecision, w2v_dense::DontAlignCols);
  if (binary) {
    std::ofstream out(filename, std::ios::binary);
    const char blank = ' ', enter = '\n';
    const int r_size = (int)(data.cols() * sizeof(RMatrixXf::Scalar));
    RMatrixXf::Index r = data.rows(), c = data.cols();
    out.write((const char*)&r, sizeof(RMatrixXf::Index));
    out.write(&blank, 1);
    out.write((const char*)&c, sizeof(RMatrixXf::Index));
    out.write(&enter, 1);
    for (auto v : vocab) {
      out.write(v->text.c_str(), (std::streamsize)v->text.size());
      out.write(&blank, 1);
      out.write((const char*)data.row((RMatrixXf::Index)v->index).data(), r_size);
      out.write(&enter, 1);
    }
  } else {
    std::ofstream out(filename);
    out << data.rows() << " " << data.cols() << std::endl;
    for (auto v : vocab) out << v->text << " " << data.row((RMatrixXf::Index)v->index).format(fmt) << std::endl;
  }
}

void Word2Vec::load_word2vec(std::string filename, bool binary) {
  if (W.rows() != (RMatrixXf::Index)vocab.size() || W.cols() != word_dim)
    W.resize((RMatrixXf::Index)vocab.size(), word_dim);
  if (binary) {
    std::ifstream in(filename, std::ios::binary);
    char ch;
    RMatrixXf::Index r = 0, c = 0;
    in.read((char*)&r, sizeof(RMatrixXf::Index));
    in.read(&ch, 1);
    in.read((char*)&c, sizeof(RMatrixXf::Index));
    in.read(&ch, 1);
    const std::streamsize r_size = (std::streamsize)(c * sizeof(RMatrixXf::Scalar));
    std::vector<char> skip((size_t)r_size);
    for (RMatrixXf::Index i = 0; i < r && in; ++i) {
      std::string text;
      in.read(&ch, 1);
      while (in && ch != ' ') {
        text += ch;
        in.read(&ch, 1);
      }
      auto it = vocab_hash.find(text);
      if (it != vocab_hash.end() && c == word_dim) in.read((char*)W.row((RMatrixXf::Index)it->second->index).data(), r_size);
      else in.read(skip.data(), r_size);
      in.read(&ch, 1);
    }
  } else {
    std::ifstream in(filename);
    std::string line, text;
    std::getline(in, line);
    size_t vsize = 0, dim = 0;
    std::istringstream hdr(line);
    hdr >> vsize >> dim;
    while (std::getline(in, line)) {
      std::istringstream iss(line);
      iss >> text;
      auto it = vocab_hash.find(text);
      if (it == vocab_hash.end()) continue;
      auto row = W.row((RMatrixXf::Index)it->second->index);
      for (size_t i = 0; i < dim && (RMatrixXf::Index)i < row.size(); ++i) iss >> row[(RMatrixXf::Index)i];
    }
  }
}
