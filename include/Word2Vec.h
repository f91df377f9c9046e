// Word2Vec.h — the reference's class API (/root/reference/Word2Vec.h:29-90),
// same members, constructor defaults and method signatures, with the training
// hot path running on an MI355X through the C-ABI in w2v_dev.h.
//
// What stays on the host (C++11): vocabulary, Huffman tree, unigram table,
// subsampling probabilities, weight init, sentence shuffling and the vector
// files — all bit-identical to the reference. What moves to HBM: W, C and
// synapses1, the table, the sample probabilities, the Huffman paths and the
// corpus as token ids; every update of train(), train_sentence_*,
// negative_sampling and hierarchical_softmax runs in the gfx950 kernels.
//
// Additive members (not in the reference) are grouped at the end.
#ifndef W2V_AMD_WORD2VEC_H
#define W2V_AMD_WORD2VEC_H

#include <cstdint>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "Word.h"
#include "w2v_dense.h"
#include "w2v_dev.h"
#include "w2v_ingest.h"

using w2v_dense::IOFormat;
using w2v_dense::RMatrixXf;
using w2v_dense::RowVectorXf;

// Drop-in compatibility with the reference header's environment
// (/root/reference/Word2Vec.h:4-24): its callers — the reference's own
// main.cpp — compile against the standard headers it includes, `using
// namespace std` / `using namespace Eigen`, Eigen::initParallel()
// (main.cpp:96) and omp_set_num_threads (main.cpp:186, declared by the
// <omp.h> Eigen pulls in under the reference's -fopenmp). Here: the same
// standard headers, both using-directives over a minimal namespace Eigen
// (initParallel is a no-op: nothing here runs Eigen's threads), and <omp.h>
// under -fopenmp. The reference's main.cpp then compiles unmodified against
// include/ (tests/test_class_host.py::test_reference_caller_compiles).
// Define W2V_NO_REFERENCE_ENVIRONMENT to keep all of this out (a translation
// unit that includes the real Eigen must include it first or define it).
#ifndef W2V_NO_REFERENCE_ENVIRONMENT
#include <algorithm>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <list>
#include <numeric>
#include <set>
#include <sstream>
#include <tuple>
#ifdef _OPENMP
#include <omp.h>
#endif
#ifndef EIGEN_WORLD_VERSION  // the real Eigen is not in this translation unit
namespace Eigen {
inline void initParallel() {}
using w2v_dense::IOFormat;
}  // namespace Eigen
#endif
using namespace std;
using namespace Eigen;
#endif

class Word2Vec {
 public:
  int iter;
  int window;
  int min_count;
  int table_size;
  int word_dim;
  int negative;  // number of negative samples
  float subsample_threshold;
  float init_alpha;
  float min_alpha;
  int num_threads;  // host threads the reference used; unused by the device path

  bool cbow_mean;
  bool phrase;
  std::string train_method;  // "hs" or "ns"
  std::string model;         // "cbow" or "sg"

  std::vector<Word*> vocab;
  std::vector<std::string> idx2word;
  std::unordered_map<std::string, WordP> vocab_hash;
  std::vector<size_t> table;

  RMatrixXf W, synapses1, C;

  std::random_device rd;
  std::mt19937 generator;
  std::uniform_int_distribution<int> distribution_window;
  std::uniform_int_distribution<int> distribution_table;
  std::uniform_real_distribution<float> uni_dis;

 public:
  ~Word2Vec(void);

  Word2Vec(int iter = 1, int window = 5, int min_count = 5, int table_size = 100000000, int word_dim = 200,
           int negative = 0, float subsample_threshold = 0.001, float init_alpha = 0.025,
           float min_alpha = 1e-6, bool cbow_mean = false, int num_threads = 1,
           std::string train_method = "hs", std::string model = "cbow");

  std::vector<std::vector<std::string>> line_docs(std::string file_name);
  void reduce_vocab();
  void create_huffman_tree();
  void make_table();
  void precalc_sampling();
  void build_vocab(std::vector<std::vector<std::string>>& sentences);
  void save_vocab(std::string vocab_filename);
  void read_vocab(std::string vocab_filename);

  void init_weights(size_t vocab_size);

  std::vector<std::vector<Word*>> build_sample(std::vector<std::vector<std::string>>& data);

  RowVectorXf& hierarchical_softmax(Word* predict_word, RowVectorXf& project_rep, RowVectorXf& project_grad,
                                    float alpha);
  RowVectorXf& negative_sampling(Word* predict_word, RowVectorXf& project_rep, RowVectorXf& project_grad,
                                 RMatrixXf& target_matrix, float alpha);
  void train_sentence_cbow(std::vector<Word*>& sentence, float alpha);
  void train_sentence_sg(std::vector<Word*>& sentence, float alpha);

  void train(std::vector<std::vector<std::string>>& sentences);

  void save_word2vec(std::string filename, const RMatrixXf& data, bool binary = false);
  void load_word2vec(std::string word2vec_filename, bool binary = false);

  // ---- additive (not in the reference) ------------------------------------
  int gpu_device = 0;        // HIP device ordinal used by the hot path
  bool replay_rng = false;   // true: the device consumes this object's own mt19937
                             // stream in the reference's draw order, on one
                             // wavefront (deterministic, equals the reference run
                             // single-threaded up to fp32 summation order)
  // parallel-schedule update policy (include/w2v_dev.h, w2v_dev_set_hot_rows ff.)
  int64_t hot_rows = W2V_HOT_AUTO;  // rows updated with device atomics: -2 auto (from the corpus), -1 all, 0 none
  int private_rows = -1;        // hottest output rows privatised in LDS: -1 as many as fit, 0 off
  int flush_centers = 0;        // workgroup centers between private-row flushes (0 = auto)
  float private_average = 8.f;  // concurrency the private rows' summed deltas are scaled to (0 = sum)
  int64_t max_waves = 0;        // wavefronts in flight (0 = as many as fit)
  int context_rows = -1;        // CBOW: hottest context rows privatised in LDS too: -1 as many as fit, 0 off
  int context_flush = 0;        // workgroup centers between context-row flushes (0 = auto)
  // BASELINE configs[4]: skip-gram NS as the shared-negatives minibatch on the
  // matrix cores (w2v_dev_set_update, W2V_UPDATE_SHARED_NEGATIVES) instead of
  // the reference's per-pair update; sg + ns only, negative <= 15, window <= 8
  bool shared_negatives = false;
  // Data-parallel replicas (BASELINE configs[3]): with >= 2 entries, train()
  // runs one full model replica per listed HIP device (a device may repeat:
  // replicas sharing one GPU share one resident corpus), each on a
  // contiguous shard of every epoch's shuffled sentence order, and exchanges
  // their updates (include/w2v_dev.h w2v_group_*: RCCL all-reduce over xGMI)
  // every sync_words in-vocab words of the largest shard (0 = auto:
  // kAutoReplicaRounds exchanges per epoch; with W2V_GROUP_AVERAGE at most one
  // per kAutoAverageWords words of a shard), overlapped with the next round's
  // training unless overlap_average is false. replica_mode: a W2V_GROUP_*
  // mode, or -1 = auto: W2V_GROUP_AVERAGE for up to kAutoAverageReplicas
  // replicas whose shards hold >= kAutoReplicaRounds x kAutoAverageWords words
  // (configs[3]'s scale: there the sum and the adaptive divisor lose 10-36
  // analogy points at two and four replicas); otherwise W2V_GROUP_SUM for two
  // replicas, W2V_GROUP_ADAPTIVE for more (the mean of a row the replicas
  // moved alike, the sum of independent moves: summing R >= 3 replicas'
  // updates overshoots the frequent rows R-fold and diverges, plain averaging
  // of short shards loses the rare rows' progress; DESIGN.md §6 has the
  // measured tables). Empty = one device (gpu_device).
  std::vector<int> gpu_devices;
  int64_t sync_words = 0;
  bool overlap_average = true;
  int replica_mode = -1;
  static const int64_t kAutoReplicaRounds = 64;  // 2 replicas within a point at 32-64 per epoch
  // ... and for the adaptive divisor (more than two replicas of short
  // shards): eight replicas of configs[3]'s shape lost 1.96 similarity points
  // at 64 exchanges per epoch, 0.13-0.64 at 96-128
  static const int64_t kAutoAdaptiveRounds = 128;
  // sync_words = 0 with replica_mode W2V_GROUP_AVERAGE: at most one exchange
  // per this many words of a shard, so each round's mean spans rows every
  // replica trained
  static const int64_t kAutoAverageWords = 4000000;
  // replica_mode auto averages at most this many replicas
  static const int64_t kAutoAverageReplicas = 4;
  bool verbose = true;       // progress line per epoch (the reference prints one
                             // every 100 sentences, Word2Vec.cpp:382-386)
  // Train on a corpus that is already token ids (no strings): ids index
  // `vocab`, sentence s spans [offsets[s], offsets[s+1]); train_words as in
  // Word2Vec.cpp:362-363 (raw tokens incl. OOV). For corpora too large for
  // vector<vector<string>>.
  void train_ids(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets, int64_t train_words);
  // Corpus files too large for vector<vector<string>> (mapped, tokenised by
  // host threads; threads <= 0 = all): format "lines" reads like line_docs
  // (Word2Vec.cpp:19-30), "text8" like the reference CLI (main.cpp:63-92,
  // 1000-token sentences). Same vocabulary (bit-exact), samples and
  // train_words as build_vocab / train on the sentences those readers return.
  void build_vocab_file(const std::string& path, const std::string& format = "lines", int threads = 0);
  void train_file(const std::string& path, const std::string& format = "lines", int threads = 0);
  // With gpu_ingest, build_vocab_file and file_samples / train_file count and
  // map the file on the GPU (include/w2v_ingest.h) instead of host threads:
  // same vocabulary, ids, offsets and train_words. The count of
  // build_vocab_file is kept for a train_file on the same file.
  bool gpu_ingest = false;
  int64_t ingest_chunk_bytes = 0;  // bytes per host -> device chunk (0 = 1 GiB)
  // build_sample of a corpus file as token ids (what train_file trains on).
  void file_samples(const std::string& path, const std::string& format, int threads, std::vector<int32_t>& ids,
                    std::vector<int64_t>& offsets, int64_t& train_words);
  // Checkpoints: W, C, synapses1, the word counter, the epochs
  // of the `iter` schedule done, the device RNG key and the generator state.
  // With checkpoint_path set, train() / train_ids() / train_file() write one
  // after every epoch ("%d" in the path = the epochs done, else overwritten).
  // After load_checkpoint the next train call starts from the restored
  // weights (no init_weights): a checkpoint taken mid-schedule (epochs done <
  // iter) runs the remaining epochs with the saved counter, key and shuffle
  // stream, i.e. continues that run (alpha follows the original schedule);
  // one taken after the whole schedule starts a new schedule on the loaded
  // weights (current_words from 0, as every train() of the reference,
  // Word2Vec.cpp:359). load_checkpoint checks every matrix's shape against
  // this object's vocab, word_dim, model and train_method and changes nothing
  // unless all of it is valid.
  std::string checkpoint_path;
  void save_checkpoint(const std::string& path);
  void load_checkpoint(const std::string& path);
  int64_t current_words() const { return cur_words_; }
  int64_t epochs_done() const { return epochs_done_; }
  // Wall seconds of each epoch of the last train call (the device epoch,
  // w2v_dev_train_epoch / the replicas' rounds; no host setup or transfers).
  std::vector<double> epoch_seconds;
  // Data-parallel replicas (gpu_devices) of the last train call: the
  // exchanges run (w2v_group_info rounds) and how far the replicas' models
  // were apart after the last one: max over replicas and matrices of
  // max |M_i - M_0| / max |M_0| (w2v_dev_model_max_diff; -1 = not measured).
  int64_t replica_rounds = 0;
  double replica_max_diff = -1.0;
  // Last device error (empty if none).
  std::string last_error;

 private:
  w2v_dev* dev_ = nullptr;
  w2v_dev_config dev_cfg_{};        // configuration dev_ was created with
  bool dev_vocab_stale_ = true;     // vocab products changed since the last upload
  int64_t cur_words_ = 0;           // current_words after the last train call
  bool resume_ = false;             // load_checkpoint: the next train continues (no init_weights)
  int64_t start_words_ = 0;         //   ... from this current_words
  int64_t resume_epochs_ = 0;       //   ... after this many epochs of the schedule
  int64_t resume_iter_ = 0;         //   ... of a schedule of this many epochs (compared with iter at train time)
  uint64_t resume_key_ = 0;         //   ... with this Philox key
  int64_t epochs_done_ = 0;         // epochs of the last train call's schedule completed
  uint64_t key_ = 0;                // Philox key of the last train call
  std::string sched_gen_;           // generator state at the start of the last train call's schedule
  std::string resume_sched_gen_;    // ... of the checkpoint's schedule (replayed to continue it)
  void write_checkpoint(const std::string& path, int64_t cw, int64_t epochs_done, uint64_t key);
  void checkpoint_epoch(int64_t cw, int64_t epochs_done, uint64_t key);
  std::string generator_state() const;
  void restore_generator(const std::string& state);
  bool continues_schedule() const;
  w2v_ingest* ingest_ = nullptr;    // gpu_ingest: the counted file ...
  std::string ingest_key_;          //   ... (path + format)
  std::vector<std::string> ingest_words_;  // its distinct words, in order of first occurrence
  std::vector<int64_t> ingest_counts_;
  void ingest_count(const std::string& path, const std::string& format);

  bool uses_C() const;
  void check_limits() const;
  void finish_vocab(std::unordered_map<std::string, int>& tally);
  void ensure_device();
  void upload_vocab_products();
  void upload_vocab_to(w2v_dev* d);
  void apply_policy(w2v_dev* d);
  void run_epochs_replicas(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets, int64_t train_words);
  void check(int rc, const char* what);
  void run_epochs(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets, int64_t train_words);
  void append_reference_draws(const std::vector<int32_t>& ids, const std::vector<int64_t>& offsets,
                              const std::vector<long>& order, std::vector<uint32_t>& stream,
                              std::vector<int64_t>& stream_off, int64_t epoch, std::vector<int32_t>* negs = nullptr);
  void train_one_sentence(std::vector<Word*>& sentence, float alpha, bool cbow);
  void apply_rows(RMatrixXf& M, int which, const std::vector<size_t>& rows, const std::vector<uint8_t>& codes,
                  RowVectorXf& x, RowVectorXf& grad, float alpha, bool hs_form);
};

#endif  // W2V_AMD_WORD2VEC_H
