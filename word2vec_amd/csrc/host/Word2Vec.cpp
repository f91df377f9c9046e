// Word2Vec.cpp — host side of the Word2Vec class API (include/Word2Vec.h).
//
// Each method keeps the reference's contract (/root/reference/Word2Vec.cpp,
// cited per method); the vocabulary products are computed by the bit-exact
// restatements in vocab_products.cpp, and every model update runs on the GPU
// through include/w2v_dev.h.
#include "Word2Vec.h"

#include <algorithm>
#include <limits>
#include <chrono>
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
  if (ingest_) w2v_ingest_destroy(ingest_);
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
  if (gpu_ingest) {
    ingest_count(path, format);
    std::unordered_map<std::string, int> tally;
    for (size_t k = 0; k < ingest_words_.size(); ++k) tally[ingest_words_[k]] = (int)ingest_counts_[k];
    finish_vocab(tally);
    return;
  }
  const w2v_corpus::File f(path);
  const w2v_corpus::Counts c = w2v_corpus::count_words(f, w2v_corpus::parse_format(format), threads);
  std::unordered_map<std::string, int> tally;
  for (const auto& wc : c.words) tally[wc.first] = (int)wc.second;
  finish_vocab(tally);
}

// Pass 1 on the GPU (w2v_ingest_count): the distinct words in order of first
// occurrence, their text read back from the mapped file at their first offset.
void Word2Vec::ingest_count(const std::string& path, const std::string& format) {
  const w2v_corpus::Format fmt = w2v_corpus::parse_format(format);
  const std::string key = format + ":" + path;
  if (ingest_ && ingest_key_ == key) return;
  if (ingest_) w2v_ingest_destroy(ingest_);
  ingest_ = nullptr;
  ingest_key_.clear();
  const w2v_corpus::File f(path);
  w2v_ingest* g = nullptr;
  check(w2v_ingest_create(gpu_device, fmt == w2v_corpus::kText8 ? W2V_INGEST_TEXT8 : W2V_INGEST_LINES,
                          ingest_chunk_bytes, &g),
        "w2v_ingest_create");
  ingest_ = g;
  check(w2v_ingest_count(g, f.data(), (int64_t)f.size()), "w2v_ingest_count");
  int64_t n_words = 0;
  check(w2v_ingest_summary(g, &n_words, nullptr, nullptr), "w2v_ingest_summary");
  std::vector<int64_t> first((size_t)n_words);
  std::vector<int32_t> len((size_t)n_words);
  ingest_counts_.assign((size_t)n_words, 0);
  check(w2v_ingest_words(g, first.data(), len.data(), ingest_counts_.data()), "w2v_ingest_words");
  ingest_words_.resize((size_t)n_words);
  for (size_t k = 0; k < (size_t)n_words; ++k) ingest_words_[k].assign(f.data() + first[k], (size_t)len[k]);
  ingest_key_ = key;
}

void Word2Vec::file_samples(const std::string& path, const std::string& format, int threads,
                            std::vector<int32_t>& ids, std::vector<int64_t>& offsets, int64_t& train_words) {
  if (gpu_ingest) {
    ingest_count(path, format);
    std::vector<int32_t> index(ingest_words_.size(), -1);
    for (size_t k = 0; k < ingest_words_.size(); ++k) {
      auto it = vocab_hash.find(ingest_words_[k]);
      if (it != vocab_hash.end()) index[k] = (int32_t)it->second->index;
    }
    const w2v_corpus::File f(path);
    check(w2v_ingest_map(ingest_, f.data(), (int64_t)f.size(), index.data(), (int64_t)index.size()), "w2v_ingest_map");
    int64_t n_ids = 0, n_sent = 0;
    check(w2v_ingest_samples_size(ingest_, &n_ids, &n_sent, &train_words), "w2v_ingest_samples_size");
    ids.resize((size_t)n_ids);
    offsets.resize((size_t)n_sent + 1);
    check(w2v_ingest_download(ingest_, ids.data(), offsets.data()), "w2v_ingest_download");
    // the samples are on the host now: free the ingest handle's device memory
    // (the resident file, the chunk work buffers, the hash table and the ids)
    // before training uploads the corpus and the model to the same device
    w2v_ingest_destroy(ingest_);
    ingest_ = nullptr;
    ingest_key_.clear();
    return;
  }
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
  check_limits();
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
  upload_vocab_to(dev_);
  dev_vocab_stale_ = false;
}

// The vocab products the kernels read (sample probabilities, table
// boundaries, Huffman CSR) onto one device handle.
void Word2Vec::upload_vocab_to(w2v_dev* d) {
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
  check(w2v_dev_upload_vocab(d, V, keep.data(), bounds.empty() ? nullptr : bounds.data(),
                             codes.empty() ? nullptr : codes.data(), points.empty() ? nullptr : points.data(),
                             off.empty() ? nullptr : off.data()),
        "w2v_dev_upload_vocab");
}

void Word2Vec::apply_policy(w2v_dev* d) {
  check(w2v_dev_set_fixed_alpha(d, 0.0f), "w2v_dev_set_fixed_alpha");
  check(w2v_dev_set_hot_rows(d, hot_rows), "w2v_dev_set_hot_rows");
  check(w2v_dev_set_private_rows(d, private_rows), "w2v_dev_set_private_rows");
  check(w2v_dev_set_private_sync(d, flush_centers, private_average), "w2v_dev_set_private_sync");
  check(w2v_dev_set_max_waves(d, max_waves), "w2v_dev_set_max_waves");
  check(w2v_dev_set_context_private(d, context_rows, context_flush), "w2v_dev_set_context_private");
  check(w2v_dev_set_update(d, shared_negatives ? W2V_UPDATE_SHARED_NEGATIVES : W2V_UPDATE_PER_PAIR),
        "w2v_dev_set_update");
}

// The draws the reference makes for one pass over `order`, in its order
// (Word2Vec.cpp:279-310 CBOW, :325-349 SG, :254-255 NS), taken from this
// object's generator, with each sentence's start recorded.
void Word2Vec::append_reference_draws(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets,
                                      const std::vector<long>& order, std::vector<uint32_t>& stream,
                                      std::vector<int64_t>& stream_off, int64_t epoch, std::vector<int32_t>* negs) {
  auto table_draw = [&]() {
    const int pos = distribution_table(generator);
    stream.push_back((uint32_t)pos);
    if (negs) negs->push_back((int32_t)table[(size_t)pos]);
  };
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
        for (int k = 0; k < negative; ++k) table_draw();
      } else {
        for (int j = lo; j < hi; ++j) {
          if (j == i) continue;
          for (int k = 0; k < negative; ++k) table_draw();
        }
      }
    }
  }
}

// The epoch loop of Word2Vec.cpp:367-395 with the model resident in HBM.
void Word2Vec::run_epochs(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets,
                          int64_t train_words) {
  if (gpu_devices.size() > 1) {
    run_epochs_replicas(ids, offsets, train_words);
    return;
  }
  ensure_device();
  upload_vocab_products();
  check(w2v_dev_upload_model(dev_, W.data(), uses_C() ? C.data() : nullptr,
                             train_method == "hs" ? synapses1.data() : nullptr),
        "w2v_dev_upload_model");
  const int64_t n = (int64_t)offsets.size() - 1;
  check(w2v_dev_upload_corpus(dev_, ids.data(), (int64_t)ids.size(), offsets.data(), n, train_words),
        "w2v_dev_upload_corpus");
  apply_policy(dev_);
  // a checkpoint taken mid-schedule continues that schedule (its counter, key
  // and shuffle stream); anything else starts one: current_words = 0 (:359)
  const bool cont = continues_schedule();
  const int first = cont ? (int)resume_epochs_ : 0;
  check(w2v_dev_set_progress(dev_, cont ? start_words_ : 0), "w2v_dev_set_progress");
  std::vector<long> sample_idx((size_t)n);
  std::iota(sample_idx.begin(), sample_idx.end(), 0);
  std::vector<std::vector<int64_t>> orders((size_t)iter);
  uint64_t key = 0;
  if (!replay_rng) key = cont ? resume_key_ : ((uint64_t)generator() << 32) | (uint64_t)generator();
  // the schedule's shuffles are cumulative (each epoch shuffles the previous
  // order) and the replay stream follows them: continuing replays the whole
  // schedule's generator from its start and trains the remaining epochs
  if (cont) restore_generator(resume_sched_gen_);
  sched_gen_ = generator_state();
  if (replay_rng) {
    std::vector<uint32_t> stream;
    std::vector<int64_t> stream_off((size_t)(n * iter), 0);
    for (int it = 0; it < iter; ++it) {
      std::shuffle(sample_idx.begin(), sample_idx.end(), generator);
      orders[(size_t)it].assign(sample_idx.begin(), sample_idx.end());
      append_reference_draws(ids, offsets, sample_idx, stream, stream_off, it);
    }
    check(w2v_dev_upload_replay(dev_, stream.data(), (int64_t)stream.size(), stream_off.data(),
                                (int64_t)stream_off.size()),
          "w2v_dev_upload_replay");
    check(w2v_dev_set_rng(dev_, W2V_RNG_REPLAY, 0), "w2v_dev_set_rng");
    check(w2v_dev_set_schedule(dev_, W2V_SCHED_SEQUENTIAL), "w2v_dev_set_schedule");
  } else {
    check(w2v_dev_set_rng(dev_, W2V_RNG_PHILOX, key), "w2v_dev_set_rng");
    check(w2v_dev_set_schedule(dev_, W2V_SCHED_PARALLEL), "w2v_dev_set_schedule");
  }
  key_ = key;
  epochs_done_ = first;
  resume_ = false;
  epoch_seconds.clear();
  for (int it = 0; it < iter; ++it) {
    if (!replay_rng) {
      std::shuffle(sample_idx.begin(), sample_idx.end(), generator);
      orders[(size_t)it].assign(sample_idx.begin(), sample_idx.end());
    }
    if (it < first) continue;  // done before the checkpoint
    w2v_dev_stats st;
    std::memset(&st, 0, sizeof(st));
    const auto t0 = std::chrono::steady_clock::now();
    check(w2v_dev_train_epoch(dev_, it, orders[(size_t)it].data(), &st), "w2v_dev_train_epoch");
    epoch_seconds.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    int64_t cw = 0;
    check(w2v_dev_get_progress(dev_, &cw), "w2v_dev_get_progress");
    epochs_done_ = it + 1;
    cur_words_ = cw;
    if (!checkpoint_path.empty()) {
      check(w2v_dev_download_model(dev_, W.data(), uses_C() ? C.data() : nullptr,
                                   train_method == "hs" ? synapses1.data() : nullptr),
            "w2v_dev_download_model");
      checkpoint_epoch(cw, it + 1, key);
    }
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

// The epoch loop of Word2Vec.cpp:367-395 over R data-parallel replicas
// (gpu_devices): every epoch's std::shuffle order is cut into R contiguous
// shards; each replica trains its shard in rounds and the replicas exchange
// their updates after every round (w2v_group_average_async: summed with RCCL
// over xGMI, or by a kernel for replicas sharing a device). The alpha schedule stays the global
// one: each replica's counter starts a round at (global words) / R with
// train_words / R as the denominator. Throughput mode (Philox) only.
void Word2Vec::run_epochs_replicas(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets,
                                   int64_t train_words) {
  if (replay_rng) throw std::runtime_error("word2vec_amd: replay_rng trains on one device (gpu_devices must be empty)");
  const size_t R = gpu_devices.size();
  const int64_t n = (int64_t)offsets.size() - 1;
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
  std::vector<w2v_dev*> reps(R, nullptr);
  w2v_group* grp = nullptr;
  auto release = [&]() {
    if (grp) w2v_group_destroy(grp);
    grp = nullptr;
    for (size_t i = reps.size(); i-- > 0;) {  // borrowers of a shared corpus before its owner
      if (reps[i]) w2v_dev_destroy(reps[i]);
      reps[i] = nullptr;
    }
  };
  try {
    const bool cont = continues_schedule();  // as run_epochs
    const int first = cont ? (int)resume_epochs_ : 0;
    const uint64_t key = cont ? resume_key_ : ((uint64_t)generator() << 32) | (uint64_t)generator();
    key_ = key;
    if (cont) restore_generator(resume_sched_gen_);  // as run_epochs: replay the schedule's shuffles
    sched_gen_ = generator_state();
    for (size_t i = 0; i < R; ++i) {
      cfg.device = gpu_devices[i];
      check(w2v_dev_create(&cfg, &reps[i]), "w2v_dev_create");
      upload_vocab_to(reps[i]);
      check(w2v_dev_upload_model(reps[i], W.data(), uses_C() ? C.data() : nullptr,
                                 train_method == "hs" ? synapses1.data() : nullptr),
            "w2v_dev_upload_model");
      size_t owner = i;  // replicas sharing a device share one resident corpus (w2v_dev_share_corpus)
      for (size_t j = 0; j < i && owner == i; ++j)
        if (gpu_devices[j] == gpu_devices[i]) owner = j;
      if (owner != i)
        check(w2v_dev_share_corpus(reps[i], reps[owner]), "w2v_dev_share_corpus");
      else
        check(w2v_dev_upload_corpus(reps[i], ids.data(), (int64_t)ids.size(), offsets.data(), n,
                                    std::max<int64_t>(1, train_words)),
              "w2v_dev_upload_corpus");
      check(w2v_dev_set_train_words(reps[i], std::max<int64_t>(1, train_words / (int64_t)R)),
            "w2v_dev_set_train_words");
      apply_policy(reps[i]);
      check(w2v_dev_set_rng(reps[i], W2V_RNG_PHILOX, key), "w2v_dev_set_rng");
      check(w2v_dev_set_schedule(reps[i], W2V_SCHED_PARALLEL), "w2v_dev_set_schedule");
    }
    check(w2v_group_create(reps.data(), (int32_t)R, nullptr, (int32_t)R, 0, &grp), "w2v_group_create");
    check(w2v_group_set_overlap(grp, overlap_average ? 1 : 0), "w2v_group_set_overlap");
    // auto: for up to kAutoAverageReplicas replicas whose
    // shards give the averaging cadence its full kAutoReplicaRounds rounds
    // (>= kAutoAverageWords words each), the plain mean — at 10 B tokens two
    // and four averaged replicas hold the single model (+6.7 / +7.1 analogy,
    // 0.0 similarity) where the sum and the adaptive divisor lose 36 and 10
    // points; otherwise the sum for two replicas and, for more, the adaptive
    // per-row divisor (the mean where the replicas moved a row alike, the sum
    // where their moves were independent: at 10 B tokens eight replicas hold
    // the single model's similarity where the plain mean loses 2.4 points)
    const bool long_shards = train_words / (int64_t)R >= kAutoReplicaRounds * kAutoAverageWords;
    const int mode = replica_mode >= 0 ? replica_mode
                     : (R <= (size_t)kAutoAverageReplicas && long_shards) ? W2V_GROUP_AVERAGE
                     : R <= 2 ? W2V_GROUP_SUM : W2V_GROUP_ADAPTIVE;
    const int64_t auto_rounds = mode == W2V_GROUP_ADAPTIVE ? kAutoAdaptiveRounds : kAutoReplicaRounds;
    check(w2v_group_set_mode(grp, mode), "w2v_group_set_mode");
    std::vector<long> sample_idx((size_t)n);
    std::iota(sample_idx.begin(), sample_idx.end(), 0);
    int64_t global = cont ? start_words_ : 0;  // the reference's current_words over all replicas (:359, :393)
    epochs_done_ = first;
    resume_ = false;
    epoch_seconds.clear();
    replica_rounds = 0;
    replica_max_diff = -1.0;
    for (int it = 0; it < iter; ++it) {
      std::shuffle(sample_idx.begin(), sample_idx.end(), generator);  // :373
      if (it < first) continue;  // done before the checkpoint
      const auto t0 = std::chrono::steady_clock::now();
      // shards and their per-sentence word counts
      std::vector<std::vector<int64_t>> shard(R), cum(R);
      int64_t largest = 0;
      for (size_t i = 0; i < R; ++i) {
        const int64_t lo = n * (int64_t)i / (int64_t)R, hi = n * (int64_t)(i + 1) / (int64_t)R;
        shard[i].assign(sample_idx.begin() + lo, sample_idx.begin() + hi);
        cum[i].assign(1, 0);
        for (int64_t s2 : shard[i]) cum[i].push_back(cum[i].back() + offsets[(size_t)s2 + 1] - offsets[(size_t)s2]);
        largest = std::max(largest, cum[i].back());
        check(w2v_dev_set_order(reps[i], shard[i].data(), (int64_t)shard[i].size()), "w2v_dev_set_order");
      }
      // auto cadence: kAutoReplicaRounds per epoch (kAutoAdaptiveRounds for
      // the adaptive divisor); plain averaging wants
      // LONG rounds — a round's mean divides the progress of every row only
      // one replica touched in it by R — so with W2V_GROUP_AVERAGE at most
      // one exchange per kAutoAverageWords words of a shard
      const int64_t avg_rounds = std::max<int64_t>(1, largest / kAutoAverageWords);
      const int64_t rounds = sync_words > 0 ? std::max<int64_t>(1, (largest + sync_words - 1) / sync_words)
                             : mode != W2V_GROUP_AVERAGE ? std::max<int64_t>(1, std::min<int64_t>(auto_rounds, largest))
                                                         : std::min<int64_t>(auto_rounds, avg_rounds);
      for (int64_t r = 0; r < rounds; ++r) {
        int64_t words = 0;
        for (size_t i = 0; i < R; ++i) {
          const int64_t m = (int64_t)shard[i].size(), lo = m * r / rounds, hi = m * (r + 1) / rounds;
          check(w2v_dev_set_progress_async(reps[i], global / (int64_t)R), "w2v_dev_set_progress_async");
          if (hi > lo) check(w2v_dev_train_slice_async(reps[i], it, lo, hi - lo), "w2v_dev_train_slice_async");
          words += cum[i][(size_t)hi] - cum[i][(size_t)lo];
        }
        check(w2v_group_average_async(grp), "w2v_group_average_async");
        global += words;
      }
      check(w2v_group_finish(grp), "w2v_group_finish");
      epoch_seconds.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      for (size_t i = 0; i < R; ++i) {
        w2v_dev_stats st;
        check(w2v_dev_read_stats(reps[i], &st), "w2v_dev_read_stats");
        if (st.nonfinite > 0)
          throw std::runtime_error("word2vec_amd: training diverged on replica " + std::to_string(i) + " (" +
                                   std::to_string(st.nonfinite) + " non-finite sigma arguments)");
      }
      epochs_done_ = it + 1;
      cur_words_ = global;
      if (!checkpoint_path.empty()) {
        check(w2v_dev_download_model(reps[0], W.data(), uses_C() ? C.data() : nullptr,
                                     train_method == "hs" ? synapses1.data() : nullptr),
              "w2v_dev_download_model");
        checkpoint_epoch(global, it + 1, key);
      }
      if (verbose) {
        std::printf("\rinit_alpha: %f  Progress: %f%% ", init_alpha, 100.0 / iter * global / train_words);
        std::fflush(stdout);
      }
    }
    cur_words_ = global;
    {
      int32_t nr = 0, loc = 0, ov = 0;
      int64_t rounds = 0;
      check(w2v_group_info(grp, &nr, &loc, &ov, &rounds), "w2v_group_info");
      replica_rounds = rounds;
      // the replicas' models after the last fold, relative to their magnitude:
      // equal up to the fp32 rounding of M + (s A - D) across the rounds
      replica_max_diff = 0.0;
      for (size_t i = 1; i < R; ++i) {
        float o[6] = {0, 0, 0, 0, 0, 0};
        check(w2v_dev_model_max_diff(reps[i], reps[0], o), "w2v_dev_model_max_diff");
        for (int k = 0; k < 3; ++k)
          if (o[3 + k] > 0.0f) replica_max_diff = std::max(replica_max_diff, (double)o[k] / (double)o[3 + k]);
          else if (o[k] > 0.0f) replica_max_diff = std::numeric_limits<double>::infinity();
      }
    }
    check(w2v_dev_download_model(reps[0], W.data(), uses_C() ? C.data() : nullptr,
                                 train_method == "hs" ? synapses1.data() : nullptr),
          "w2v_dev_download_model");
    if (verbose) std::printf("\n");
  } catch (...) {
    release();
    throw;
  }
  release();
}

// The reference accepts any window / negative / word_dim (Word2Vec.cpp:254,
// 285, 335); the kernels have a range (w2v_dev_limits). Checked before any
// corpus work, naming the member.
void Word2Vec::check_limits() const {
  int32_t md = 0, mw = 0, mn = 0, smw = 0, smn = 0;
  (void)w2v_dev_limits(&md, &mw, &mn, &smw, &smn);
  auto bad = [](const std::string& what) { throw std::invalid_argument("word2vec_amd: " + what); };
  if (word_dim < 1 || word_dim > md) bad("word_dim must be in [1, " + std::to_string(md) + "] on the GPU path");
  if (window < 0 || window > mw) bad("window must be in [0, " + std::to_string(mw) + "] on the GPU path");
  if (negative < 0 || negative > mn) bad("negative must be in [0, " + std::to_string(mn) + "] on the GPU path");
  int32_t sdim = 0;
  (void)w2v_dev_shared_limits(&sdim, nullptr, nullptr);
  if (shared_negatives && (window > smw || negative > smn || word_dim > sdim))
    bad("shared_negatives needs window <= " + std::to_string(smw) + ", negative <= " + std::to_string(smn) +
        " and word_dim <= " + std::to_string(sdim));
  // -1 (auto) or one of the modes w2v_group_set_mode takes; SPLIT / SATURATION
  // need per-row divisors the class does not compute (checked
  // before any replica is created)
  if (replica_mode < -1 || replica_mode > W2V_GROUP_ADAPTIVE)
    bad("replica_mode must be -1 (auto) or W2V_GROUP_SUM .. W2V_GROUP_ADAPTIVE (0 .. " +
        std::to_string(W2V_GROUP_ADAPTIVE) + ")");
}

// Word2Vec.cpp:356-396.
void Word2Vec::train(std::vector<std::vector<std::string>>& sentences) {
  check_limits();
  if (!resume_) init_weights(vocab.size());
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
  check_limits();
  if (!resume_) init_weights(vocab.size());
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
// device with the caller's alpha. Only the rows the update can touch cross
// PCIe (the model stays resident between calls): W and C rows of the
// sentence's words and of its negatives, and the synapses1 rows on the
// sentence words' Huffman paths — O(touched rows x dim) per call, as the
// reference's own update, instead of the whole V x dim model.
void Word2Vec::train_one_sentence(std::vector<Word*>& sentence, float alpha, bool cbow) {
  const std::string saved = model;
  model = cbow ? "cbow" : "sg";
  try {
    std::vector<int32_t> ids;
    for (Word* w : sentence) ids.push_back((int32_t)w->index);
    std::vector<int64_t> off{0, (int64_t)ids.size()};
    ensure_device();
    upload_vocab_products();
    std::vector<uint32_t> stream;
    std::vector<int64_t> soff(1, 0);
    std::vector<int32_t> negs;
    append_reference_draws(ids, off, std::vector<long>{0}, stream, soff, 0, &negs);
    // the touched rows, sorted and unique
    std::vector<int32_t> wc(ids);
    wc.insert(wc.end(), negs.begin(), negs.end());
    std::sort(wc.begin(), wc.end());
    wc.erase(std::unique(wc.begin(), wc.end()), wc.end());
    std::vector<int32_t> nodes;
    if (train_method == "hs") {
      for (int32_t w : ids)
        for (size_t p : vocab[(size_t)w]->points) nodes.push_back((int32_t)p);
      std::sort(nodes.begin(), nodes.end());
      nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
    }
    const bool has_c = uses_C() && C.size() > 0;
    const size_t d = (size_t)word_dim;
    std::vector<float> buf(std::max(wc.size(), nodes.size()) * d);
    auto move_rows = [&](int which, RMatrixXf& M, const std::vector<int32_t>& rows, bool up) {
      if (rows.empty()) return;
      if (up)
        for (size_t k = 0; k < rows.size(); ++k) std::memcpy(&buf[k * d], M.row((w2v_dense::Index)rows[k]).data(), d * 4);
      check(up ? w2v_dev_upload_rows(dev_, which, rows.data(), (int64_t)rows.size(), buf.data())
               : w2v_dev_download_rows(dev_, which, rows.data(), (int64_t)rows.size(), buf.data()),
            up ? "w2v_dev_upload_rows" : "w2v_dev_download_rows");
      if (!up)
        for (size_t k = 0; k < rows.size(); ++k) std::memcpy(M.row((w2v_dense::Index)rows[k]).data(), &buf[k * d], d * 4);
    };
    move_rows(0, W, wc, true);
    if (has_c) move_rows(1, C, wc, true);
    if (train_method == "hs") move_rows(2, synapses1, nodes, true);
    check(w2v_dev_upload_corpus(dev_, ids.data(), (int64_t)ids.size(), off.data(), 1,
                                std::max<int64_t>(1, (int64_t)ids.size())),
          "w2v_dev_upload_corpus");
    check(w2v_dev_upload_replay(dev_, stream.data(), (int64_t)stream.size(), soff.data(), 1),
          "w2v_dev_upload_replay");
    check(w2v_dev_set_rng(dev_, W2V_RNG_REPLAY, 0), "w2v_dev_set_rng");
    check(w2v_dev_set_schedule(dev_, W2V_SCHED_SEQUENTIAL), "w2v_dev_set_schedule");
    check(w2v_dev_set_fixed_alpha(dev_, alpha), "w2v_dev_set_fixed_alpha");
    check(w2v_dev_train_epoch(dev_, 0, nullptr, nullptr), "w2v_dev_train_epoch");
    check(w2v_dev_set_fixed_alpha(dev_, 0.0f), "w2v_dev_set_fixed_alpha");
    move_rows(0, W, wc, false);
    if (has_c) move_rows(1, C, wc, false);
    if (train_method == "hs") move_rows(2, synapses1, nodes, false);
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

// ---------------------------------------------------------------------------
// Checkpoints (additive; SURVEY.md §5: the reference saves only the final
// vectors, Word2Vec.cpp:398-438): W, C, synapses1, the word counter
// (current_words, Word2Vec.cpp:359,393), the epochs of the schedule done, the
// iter they belong to, the Philox key and the generator state, with the
// vocabulary's size and a hash of its words to catch a mismatched resume.
// Semantics: include/Word2Vec.h (checkpoint_path, load_checkpoint).
// ---------------------------------------------------------------------------
namespace {

const char kCkptMagic[8] = {'W', '2', 'V', 'C', 'K', 'P', 'T', '2'};

uint64_t vocab_hash64(const std::vector<Word*>& vocab) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a over "text\0count\0" in vocab order
  for (const Word* w : vocab) {
    for (char c : w->text + std::string(1, '\0') + std::to_string(w->count) + std::string(1, '\0')) {
      h ^= (uint8_t)c;
      h *= 1099511628211ull;
    }
  }
  return h;
}

void write_matrix(std::ofstream& out, const RMatrixXf& M) {
  const int64_t r = M.rows(), c = M.cols();
  out.write((const char*)&r, 8);
  out.write((const char*)&c, 8);
  if (r * c > 0) out.write((const char*)M.data(), (std::streamsize)(r * c * 4));
}

// A matrix of exactly `rows` x `cols` (rows == 0: an empty matrix, any cols).
void read_matrix(std::ifstream& in, RMatrixXf& M, int64_t rows, int64_t cols, const char* name) {
  int64_t r = 0, c = 0;
  in.read((char*)&r, 8);
  in.read((char*)&c, 8);
  if (!in || r < 0 || c < 0 || r * c > ((int64_t)1 << 40)) throw std::runtime_error("checkpoint: bad matrix header");
  const bool ok = rows == 0 ? r * c == 0 : (r == rows && c == cols);
  if (!ok)
    throw std::runtime_error(std::string("checkpoint: ") + name + " is " + std::to_string(r) + " x " +
                             std::to_string(c) + ", this object needs " + std::to_string(rows) + " x " +
                             std::to_string(rows ? cols : 0));
  M.resize((w2v_dense::Index)r, (w2v_dense::Index)c);
  if (r * c > 0) in.read((char*)M.data(), (std::streamsize)(r * c * 4));
  if (!in) throw std::runtime_error("checkpoint: truncated matrix");
}

}  // namespace

void Word2Vec::write_checkpoint(const std::string& path, int64_t cw, int64_t epochs_done, uint64_t key) {
  std::ofstream out(path, std::ios::binary);
  if (!out) throw std::runtime_error("checkpoint: cannot write " + path);
  out.write(kCkptMagic, 8);
  const int64_t hdr[2] = {(int64_t)vocab.size(), (int64_t)word_dim};
  const uint64_t vh = vocab_hash64(vocab);
  const int64_t pos[3] = {cw, epochs_done, (int64_t)iter};
  out.write((const char*)hdr, 16);
  out.write((const char*)&vh, 8);
  out.write((const char*)pos, 24);
  out.write((const char*)&key, 8);
  for (const std::string& g : {generator_state(), sched_gen_}) {
    const int64_t gl = (int64_t)g.size();
    out.write((const char*)&gl, 8);
    out.write(g.data(), (std::streamsize)gl);
  }
  write_matrix(out, W);
  write_matrix(out, C);
  write_matrix(out, synapses1);
  if (!out) throw std::runtime_error("checkpoint: write failed for " + path);
}

// After epoch `epochs_done` of a train call (checkpoint_path set; the host
// matrices hold that epoch's model).
void Word2Vec::checkpoint_epoch(int64_t cw, int64_t epochs_done, uint64_t key) {
  std::string path = checkpoint_path;
  const size_t p = path.find("%d");
  if (p != std::string::npos) path.replace(p, 2, std::to_string(epochs_done));
  write_checkpoint(path, cw, epochs_done, key);
}

std::string Word2Vec::generator_state() const {
  std::ostringstream gs;
  gs << generator;
  return gs.str();
}

void Word2Vec::restore_generator(const std::string& state) {
  std::istringstream gs(state);
  gs >> generator;
  if (!gs) throw std::runtime_error("word2vec_amd: bad saved generator state");
}

void Word2Vec::save_checkpoint(const std::string& path) { write_checkpoint(path, cur_words_, epochs_done_, key_); }

// Whether the next train call continues a loaded checkpoint's schedule: one
// taken mid-schedule (0 < epochs done < its iter) of a schedule as long as
// this object's iter NOW (decided at train time: iter may change after the
// load).
bool Word2Vec::continues_schedule() const {
  return resume_ && resume_epochs_ > 0 && resume_iter_ == iter && resume_epochs_ < iter;
}

void Word2Vec::load_checkpoint(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) throw std::runtime_error("checkpoint: cannot read " + path);
  char magic[8];
  in.read(magic, 8);
  if (!in || std::memcmp(magic, "W2VCKPT", 7) != 0) throw std::runtime_error("checkpoint: not a word2vec_amd checkpoint");
  // version 1 (round 2): V, d, vocab hash, current_words, the generator, the
  // matrices: no schedule position, so it loads as a whole-schedule checkpoint
  // (the next train starts a new schedule on its weights)
  const int version = magic[7] == '1' ? 1 : magic[7] == kCkptMagic[7] ? 2 : 0;
  if (version == 0)
    throw std::runtime_error(std::string("checkpoint: unknown checkpoint version '") + magic[7] + "' (this build reads 1 and 2)");
  int64_t V = 0, d = 0, cw = 0, ep = 0, it = 1, gl = 0;
  uint64_t vh = 0, key = 0;
  in.read((char*)&V, 8);
  in.read((char*)&d, 8);
  in.read((char*)&vh, 8);
  in.read((char*)&cw, 8);
  if (version >= 2) {
    in.read((char*)&ep, 8);
    in.read((char*)&it, 8);
    in.read((char*)&key, 8);
  }
  if (!in || V != (int64_t)vocab.size() || d != word_dim || vh != vocab_hash64(vocab))
    throw std::runtime_error("checkpoint: vocabulary or word_dim differs from this object's");
  if (cw < 0 || ep < 0 || it < 1 || ep > it) throw std::runtime_error("checkpoint: bad schedule position");
  std::string gstate[2];  // the generator now, and at the start of the checkpoint's schedule
  std::mt19937 gen;
  for (int k = 0; k < (version >= 2 ? 2 : 1); ++k) {
    in.read((char*)&gl, 8);
    if (!in || gl < 0 || gl > (1 << 20)) throw std::runtime_error("checkpoint: bad generator state");
    gstate[k].assign((size_t)gl, '\0');
    if (gl > 0) in.read(&gstate[k][0], (std::streamsize)gl);
    if (k == 1 && gl == 0 && in) continue;  // saved before any train call: no schedule yet
    std::istringstream gs(gstate[k]);
    gs >> gen;
    if (!in || !gs) throw std::runtime_error("checkpoint: bad generator state");
  }
  {
    std::istringstream gs(gstate[0]);
    gs >> gen;
  }
  // every matrix is read into a temporary and checked against the shapes this
  // object trains (init_weights): W V x d; C V x d when uses_C(), else empty;
  // synapses1 (V-1) x d for hs, else empty
  RMatrixXf w, c, s1;
  read_matrix(in, w, V, d, "W");
  read_matrix(in, c, uses_C() ? V : 0, d, "C");
  read_matrix(in, s1, train_method == "hs" ? std::max<int64_t>(V - 1, 0) : 0, d, "synapses1");
  if (V > 0 && w.rows() == 0) throw std::runtime_error("checkpoint: saved before init_weights (W is empty)");
  // commit
  W = std::move(w);
  C = std::move(c);
  synapses1 = std::move(s1);
  generator = gen;
  cur_words_ = cw;
  start_words_ = cw;
  epochs_done_ = ep;
  key_ = key;
  // a mid-schedule checkpoint continues its schedule if iter still matches when train runs
  resume_epochs_ = ep;
  resume_iter_ = it;
  resume_key_ = key;
  resume_sched_gen_ = gstate[1];
  sched_gen_ = gstate[1];
  resume_ = true;
}
