/*
 * w2v_model.h — a C bridge over the C++ Word2Vec class (include/Word2Vec.h),
 * for FFI callers (Python ctypes in tests/, cgo/JNI-style bindings). Each call
 * maps onto one class member of the reference API (Word2Vec.h:61-90); no
 * exception crosses it: failures return non-zero and set w2v_model_last_error.
 * which: 0 = W, 1 = C, 2 = synapses1.
 */
#ifndef W2V_MODEL_H
#define W2V_MODEL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct w2v_model w2v_model;

/* Word2Vec(iter, window, min_count, table_size, word_dim, negative, subsample_threshold,
 *          init_alpha, min_alpha, cbow_mean, num_threads, train_method, model) */
w2v_model* w2v_model_new(int32_t iter, int32_t window, int32_t min_count, int32_t table_size, int32_t word_dim,
                         int32_t negative, float subsample_threshold, float init_alpha, float min_alpha,
                         int32_t cbow_mean, int32_t num_threads, const char* train_method, const char* model);
void w2v_model_free(w2v_model* m);
const char* w2v_model_last_error(w2v_model* m);
void w2v_model_seed(w2v_model* m, uint32_t seed);               /* generator.seed(seed) */
void w2v_model_options(w2v_model* m, int32_t gpu_device, int32_t replay_rng, int32_t verbose);
/* Parallel-schedule update policy (Word2Vec.h additive members; include/w2v_dev.h). */
void w2v_model_update_policy(w2v_model* m, int64_t hot_rows, int32_t private_rows, int32_t flush_centers,
                             float private_average, int64_t max_waves);
/* CBOW context-row privatisation (Word2Vec.h context_rows / context_flush; w2v_dev_set_context_private). */
void w2v_model_context_policy(w2v_model* m, int32_t context_rows, int32_t context_flush);
/* Word2Vec::shared_negatives (configs[4] minibatch skip-gram; include/w2v_dev.h w2v_dev_set_update). */
void w2v_model_set_shared_negatives(w2v_model* m, int32_t on);
/* Word2Vec::gpu_devices / sync_words / overlap_average: n >= 2 devices train
 * data-parallel replicas (a device may repeat); n < 2 = one device. */
void w2v_model_replicas(w2v_model* m, const int32_t* devices, int32_t n, int64_t sync_words, int32_t overlap);
/* Word2Vec::replica_mode (a W2V_GROUP_* mode of include/w2v_dev.h). */
void w2v_model_replica_mode(w2v_model* m, int32_t mode);
/* Word2Vec::gpu_ingest / ingest_chunk_bytes: count and map corpus files on the
 * GPU (include/w2v_ingest.h) in build_vocab_file / file_samples / train_file. */
void w2v_model_set_gpu_ingest(w2v_model* m, int32_t on, int64_t chunk_bytes);

/* Sentences as text: one per line, whitespace-separated tokens (line_docs format). */
int w2v_model_build_vocab(w2v_model* m, const char* text, int64_t len);
int w2v_model_train(w2v_model* m, const char* text, int64_t len);
int w2v_model_train_ids(w2v_model* m, const int32_t* ids, const int64_t* offsets, int64_t n_sent,
                        int64_t train_words);
int w2v_model_init_weights(w2v_model* m);
/* Corpus files (Word2Vec::build_vocab_file / train_file / file_samples):
 * format "lines" (line_docs) or "text8" (the reference CLI's reader); threads
 * <= 0 = all host threads. w2v_model_file_samples tokenises the file and keeps
 * the result in the handle; w2v_model_copy_samples copies it out (ids:
 * *n_tokens int32, offsets: *n_sentences + 1 int64). */
int w2v_model_build_vocab_file(w2v_model* m, const char* path, const char* format, int32_t threads);
int w2v_model_train_file(w2v_model* m, const char* path, const char* format, int32_t threads);
int w2v_model_file_samples(w2v_model* m, const char* path, const char* format, int32_t threads, int64_t* n_tokens,
                           int64_t* n_sentences, int64_t* train_words);
int w2v_model_copy_samples(w2v_model* m, int32_t* ids, int64_t* offsets);

/* Word introspection: an index outside [0, vocab_size) returns NULL / -1 /
 * NaN / non-zero and sets last_error. */
int64_t w2v_model_vocab_size(w2v_model* m);
const char* w2v_model_word(w2v_model* m, int64_t i);
int64_t w2v_model_word_count(w2v_model* m, int64_t i);
float w2v_model_sample_probability(w2v_model* m, int64_t i);
int64_t w2v_model_path_length(w2v_model* m, int64_t i);
int w2v_model_path(w2v_model* m, int64_t i, uint8_t* codes, int32_t* points);
int64_t w2v_model_table_length(w2v_model* m);
int w2v_model_table(w2v_model* m, uint32_t* out);

int64_t w2v_model_rows(w2v_model* m, int32_t which);
int w2v_model_get_matrix(w2v_model* m, int32_t which, float* out);
/* in: rows x cols dense floats; cols must equal word_dim (non-zero return otherwise). */
int w2v_model_set_matrix(w2v_model* m, int32_t which, const float* in, int64_t rows, int64_t cols);

/* train_sentence_sg / train_sentence_cbow on one sentence of vocab indices. */
int w2v_model_train_sentence(w2v_model* m, const int32_t* ids, int64_t n, float alpha, int32_t cbow);
/* negative_sampling (which = 0 or 1) / hierarchical_softmax for word `word`. */
int w2v_model_negative_sampling(w2v_model* m, int64_t word, float* x, float* grad, int32_t which, float alpha);
int w2v_model_hierarchical_softmax(w2v_model* m, int64_t word, float* x, float* grad, float alpha);

int w2v_model_save(w2v_model* m, const char* path, int32_t which, int32_t binary);
int w2v_model_load(w2v_model* m, const char* path, int32_t binary);
int w2v_model_save_vocab(w2v_model* m, const char* path);
/* Word2Vec::save_checkpoint / load_checkpoint (W, C, synapses1, current_words,
 * generator state; the next train continues from them) and current_words(). */
int w2v_model_save_checkpoint(w2v_model* m, const char* path);
int w2v_model_load_checkpoint(w2v_model* m, const char* path);
/* Word2Vec::checkpoint_path: a checkpoint after every epoch of train ("" = off;
 * "%d" = the epochs done); epochs of the last train call's schedule done. */
int w2v_model_set_checkpoint_path(w2v_model* m, const char* path);
int64_t w2v_model_epochs_done(w2v_model* m);
/* Word2Vec::epoch_seconds[i] of the last train call (-1 when i is out of range). */
double w2v_model_epoch_seconds(w2v_model* m, int64_t i);
int64_t w2v_model_current_words(w2v_model* m);
/* Word2Vec::replica_rounds / replica_max_diff of the last train call. */
int64_t w2v_model_replica_rounds(w2v_model* m);
double w2v_model_replica_max_diff(w2v_model* m);
int w2v_model_read_vocab(w2v_model* m, const char* path);
/* Word2Vec::create_huffman_tree / make_table / precalc_sampling
 * (Word2Vec.h:70-72; Word2Vec.cpp:32-130): the vocabulary products
 * build_vocab makes (:162-168), for a vocab read with read_vocab. */
int w2v_model_create_huffman_tree(w2v_model* m);
int w2v_model_make_table(w2v_model* m);
int w2v_model_precalc_sampling(w2v_model* m);

#ifdef __cplusplus
}
#endif
#endif /* W2V_MODEL_H */
