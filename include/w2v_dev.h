/*
 * w2v_dev.h — the C-ABI drop-in boundary between the host Word2Vec class and
 * the gfx950 (MI355X) training kernels.
 *
 * The reference (lache/word2vec) has no FFI: its hot path is the member
 * functions of class Word2Vec (/root/reference/Word2Vec.h:29-90) running an
 * OpenMP Hogwild loop over Eigen rows (Word2Vec.cpp:232-396). This header is
 * the thin C layer that host code behind the same class API calls instead of
 * that loop. Every entry point uses plain pointers and sizes (no C++/torch
 * types), returns W2V_OK or an error code, never throws, and records a
 * human-readable message retrievable with w2v_dev_last_error().
 *
 * Threading: one handle is used from one host thread at a time. Functions are
 * synchronous unless their name ends in _async; _async work is ordered on the
 * handle's HIP stream (w2v_dev_set_stream).
 *
 * Device layout (HBM): W, C and synapses1 are row-major fp32 with a row pitch
 * of w2v_dev_row_pitch floats (64 x the instantiated floats per lane covering
 * word_dim: 256-B aligned rows, zero padding; a per-pair kernel lane
 * owns elements lane + 64 v of a row, the shared-negatives kernel's wave w of
 * n the columns [pitch/n w, pitch/n (w+1))); the unigram table is
 * uint32[table_size]; sample probabilities fp32[V]; Huffman paths are CSR
 * (uint8 codes, int32 points, int64 offsets); the corpus is int32 token ids
 * with int64 sentence offsets.
 */
#ifndef W2V_DEV_H
#define W2V_DEV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define W2V_OK 0
#define W2V_ERR_ARG 1         /* invalid argument / size */
#define W2V_ERR_HIP 2         /* a HIP runtime call failed */
#define W2V_ERR_STATE 3       /* call out of order (e.g. train before upload) */
#define W2V_ERR_UNSUPPORTED 4 /* configuration outside the kernels' range */
#define W2V_ERR_DIVERGED 5    /* training produced non-finite values (w2v_dev_stats.nonfinite) */
#define W2V_ERR_COMM 6        /* an RCCL call failed (w2v_group_*) */

/* RNG modes for the training kernels. */
#define W2V_RNG_PHILOX 0 /* counter-based Philox4x32-10 per (epoch, sentence, position, slot, k) */
#define W2V_RNG_REPLAY 1 /* consume a host-recorded stream in the reference's draw order */

/* Schedules. */
#define W2V_SCHED_PARALLEL 0   /* one wavefront per sentence, Hogwild across sentences */
#define W2V_SCHED_SEQUENTIAL 1 /* one wavefront walks the sentences in order: deterministic */

/* Update formulations (w2v_dev_set_update). */
#define W2V_UPDATE_PER_PAIR 0         /* the reference's: each (center, context) pair its own NS/HS call */
#define W2V_UPDATE_SHARED_NEGATIVES 1 /* minibatch SGNS: one window's contexts x (center + shared
                                         negatives) as dense MFMA GEMMs (BASELINE configs[4]) */

typedef struct w2v_dev w2v_dev; /* opaque handle */

/* Mirrors the Word2Vec constructor arguments that shape the hot path
 * (Word2Vec.h:64-66; members Word2Vec.h:32-46). */
typedef struct w2v_dev_config {
  int32_t word_dim;  /* Word2Vec::word_dim  (Word2Vec.h:36)                      */
  int32_t window;    /* Word2Vec::window    (Word2Vec.h:33), w2v_dev_limits      */
  int32_t negative;  /* Word2Vec::negative  (Word2Vec.h:37), 0 disables NS       */
  int32_t hs;        /* train_method == "hs" (Word2Vec.cpp:162,206,342,304)       */
  int32_t cbow;      /* model == "cbow"     (Word2Vec.cpp:387-390)               */
  int32_t cbow_mean; /* Word2Vec::cbow_mean (Word2Vec.h:43)                      */
  int32_t iter;      /* Word2Vec::iter      (Word2Vec.h:32), alpha schedule      */
  float init_alpha;  /* Word2Vec::init_alpha (Word2Vec.h:39)                     */
  float min_alpha;   /* Word2Vec::min_alpha  (Word2Vec.h:40)                     */
  int64_t table_size;/* Word2Vec::table_size (Word2Vec.h:35)                     */
  int32_t device;    /* HIP device ordinal; -1 = the calling thread's current    */
  int32_t reserved;
} w2v_dev_config;

/* Counters accumulated by the kernels (reset with w2v_dev_reset_stats). */
typedef struct w2v_dev_stats {
  int64_t words;     /* in-vocab tokens consumed: the reference's current_words
                        increments (Word2Vec.cpp:392-393)                        */
  int64_t centers;   /* centers kept by subsampling (Word2Vec.cpp:282,332)       */
  int64_t contexts;  /* SG: (center, context) pairs; CBOW: unique context rows   */
  int64_t targets;   /* output rows updated: NS targets + HS path nodes          */
  int64_t draws;     /* unigram-table draws (Word2Vec.cpp:255)                   */
  int64_t sentences; /* sentences processed                                      */
  int64_t nonfinite; /* sigma arguments (row . input) that were not finite: the
                        model diverged. w2v_dev_train_epoch returns
                        W2V_ERR_DIVERGED when its epoch raised this count;
                        _async callers check it with w2v_dev_read_stats          */
} w2v_dev_stats;

/* Library / error. */
const char* w2v_dev_version(void);
const char* w2v_dev_last_error(void); /* thread-local message of the last failure */
/* The experiment environment variables (W2V_SEG_LEN, W2V_DEBUG_*, W2V_SN_*)
 * this handle read at w2v_dev_create, as "NAME=value ..." ("" when none was
 * set). They are read once there, never per launch. */
const char* w2v_dev_knobs(w2v_dev* h);

/* The kernels' range of the reference's unbounded hyper-parameters
 * (Word2Vec.cpp:254, 285, 335 accept any window / negative): word_dim <= 2048,
 * window <= 4096, negative <= 4096 (w2v_dev_create returns
 * W2V_ERR_UNSUPPORTED beyond them). Negatives past 63 are drawn and
 * deduplicated 64 at a time, CBOW windows past 127 are walked from the
 * sentence; both deduplications grow with the square of the count, so the
 * range stops where it was measured (profiles/r05b_4_limits_cost_probe.log,
 * d 64, one MI355X): per target row 6.4 ns at negative 64, 13.5 ns at 1024,
 * 46 ns at 4096; CBOW per target 0.49 us at window 128, 4.5 us at 1024,
 * 5.8 us at 2048 (2 window context rows per center). The shared-negatives
 * update: window <= 8, negative <= 15 (its 16 x 16 MFMA tiles hold a window's
 * <= 16 inputs and <= 16 outputs), word_dim <= 1024 (w2v_dev_shared_limits).
 * Callers check these up front (Word2Vec::train, the CLI) to fail before any
 * corpus work, naming the reference's member / flag. Any pointer may be NULL. */
int w2v_dev_limits(int32_t* max_dim, int32_t* max_window, int32_t* max_negative, int32_t* shared_max_window,
                   int32_t* shared_max_negative);
/* The shared-negatives update's range (W2V_UPDATE_SHARED_NEGATIVES): rows of
 * 64 x {1..8, 10, 12, 14, 16} floats (word_dim <= 1024), window <= 8,
 * negative <= 15. Any pointer may be NULL. */
int w2v_dev_shared_limits(int32_t* max_dim, int32_t* max_window, int32_t* max_negative);

/* Replaces: the Word2Vec ctor's device-relevant state (Word2Vec.cpp:12-17). */
int w2v_dev_create(const w2v_dev_config* cfg, w2v_dev** out);
void w2v_dev_destroy(w2v_dev* h);

/* Stream the handle enqueues on (a hipStream_t; NULL = a private stream). */
int w2v_dev_set_stream(w2v_dev* h, void* hip_stream);
/* RNG mode + Philox key. Replaces: generator/distribution members (Word2Vec.h:55-59). */
int w2v_dev_set_rng(w2v_dev* h, int32_t rng_mode, uint64_t seed);
int w2v_dev_set_schedule(w2v_dev* h, int32_t schedule);

/* Replaces: the products of build_vocab (Word2Vec.cpp:132-169) consumed by the
 * hot path — Word::sample_probability (precalc_sampling :115-130), the unigram
 * table (make_table :81-113) given as V+1 first-index boundaries of the
 * monotone table (NULL when negative == 0), and Word::codes/points
 * (create_huffman_tree :32-79) as CSR (NULL when hs == 0). */
int w2v_dev_upload_vocab(w2v_dev* h, int64_t vocab_size, const float* sample_probability,
                         const int64_t* table_bounds, const uint8_t* codes,
                         const int32_t* points, const int64_t* code_offsets);
/* Alternative to table_bounds: the expanded table (Word2Vec.h:51), n == table_size. */
int w2v_dev_upload_table(w2v_dev* h, const uint32_t* table, int64_t n);

/* Replaces: the W / C / synapses1 members (Word2Vec.h:53) and init_weights'
 * result (Word2Vec.cpp:198-210). Host arrays are dense rows of word_dim floats:
 * W and C have V rows, synapses1 V-1. NULL skips a matrix. */
int w2v_dev_upload_model(w2v_dev* h, const float* W, const float* C, const float* syn1);
int w2v_dev_download_model(w2v_dev* h, float* W, float* C, float* syn1);
/* How far two handles' resident models are apart: out[k] = max |A_k - B_k|
 * and out[3 + k] = max |A_k| for k = W, C, synapses1 (0 for an absent one; a
 * NaN in either counts as infinitely apart). The handles may sit on
 * different devices (b's matrix is staged on a's). No reference counterpart:
 * it checks that the replicas of a group hold one model, up to the fp32
 * rounding of their folds, after the last exchange. */
int w2v_dev_model_max_diff(w2v_dev* a, w2v_dev* b, float out[6]);
/* Row-sparse transfers: rows[k] of matrix `which` (0 = W, 1 = C, 2 =
 * synapses1) <-> data[k * word_dim .. +word_dim) (host, dense). The per-call
 * methods (Word2Vec::train_sentence_*, Word2Vec.h:83-84) move only the rows a
 * sentence's update can touch instead of the whole model. The first call
 * allocates the resident model (its other rows are not initialised). */
int w2v_dev_upload_rows(w2v_dev* h, int32_t which, const int32_t* rows, int64_t n, const float* data);
int w2v_dev_download_rows(w2v_dev* h, int32_t which, const int32_t* rows, int64_t n, float* data);
/* Train on caller-owned device matrices instead (e.g. torch tensors that an
 * RCCL all-reduce also touches): rows of `pitch` floats (pitch % 4 == 0,
 * pitch >= w2v_dev_row_pitch, 16-B aligned bases), padding columns zero
 * (the kernels read and write whole rows of w2v_dev_row_pitch floats and keep
 * the padding zero). NULL for a matrix the configuration does not use. The
 * handle never frees them. */
int w2v_dev_bind_model(w2v_dev* h, float* dW, float* dC, float* dsyn1, int64_t pitch);
/* The smallest row pitch (floats) the kernels accept: 64 x the instantiated
 * floats per lane covering word_dim (d 300 -> 320, d 700 -> 768). The
 * library-owned matrices use it. */
int w2v_dev_row_pitch(w2v_dev* h, int64_t* pitch);
/* Device pointers and row pitch (floats) of the resident matrices, for
 * collectives (RCCL model averaging) on the caller's side. */
int w2v_dev_model_layout(w2v_dev* h, float** dW, float** dC, float** dsyn1, int64_t* pitch);

/* Replaces: build_sample's vector<vector<Word*>> (Word2Vec.cpp:212-230) and
 * train_words (:362-363, raw tokens incl. OOV, drives the alpha schedule). */
int w2v_dev_upload_corpus(w2v_dev* h, const int32_t* ids, int64_t n_tokens,
                          const int64_t* sent_offsets, int64_t n_sentences,
                          int64_t train_words);
/* Train on another handle's corpus (same device, same vocab) without a copy:
 * replicas sharing one GPU (Word2Vec::gpu_devices with a repeated device)
 * each train their own order slices of ONE resident corpus (configs[3]'s 10 B
 * tokens are 40 GB: eight copies would not fit one GPU). The corpus is
 * reference-counted: destroying `src`, or uploading / adopting / sharing a new
 * corpus into it, leaves h's copy resident until h lets go too. h keeps its
 * own order buffer and statistics copy. */
int w2v_dev_share_corpus(w2v_dev* h, w2v_dev* src);
/* Replay mode: recorded draws in the reference's order (u per token; window
 * shrink per kept token; table positions per NS call) and their start offset
 * per [epoch * n_sentences + sentence]. */
int w2v_dev_upload_replay(w2v_dev* h, const uint32_t* stream, int64_t n,
                          const int64_t* stream_offsets, int64_t n_offsets);

/* The reference's shared current_words counter (Word2Vec.cpp:359,393). */
int w2v_dev_set_progress(w2v_dev* h, int64_t current_words);
int w2v_dev_get_progress(w2v_dev* h, int64_t* current_words);
/* The same, enqueued on the handle's stream (ordered between training slices). */
int w2v_dev_set_progress_async(w2v_dev* h, int64_t current_words);
/* Replace train_words (Word2Vec.cpp:362-363), the denominator of the alpha
 * schedule (:379-380). A replica that trains 1/N of the corpus with its
 * counter at (global words) / N follows the global schedule with
 * train_words = (global raw tokens) / N. */
int w2v_dev_set_train_words(w2v_dev* h, int64_t train_words);

/* Replaces: one iteration of train()'s epoch loop (Word2Vec.cpp:371-395):
 * the sentences are visited in `order` (host array of n_sentences sentence
 * ids — the std::shuffle result; NULL = identity), alpha follows the
 * reference schedule from the device progress counter, and every sentence is
 * trained by train_sentence_sg/cbow semantics (:273-353). Synchronous; adds
 * this epoch's counters to *stats when stats != NULL. */
int w2v_dev_train_epoch(w2v_dev* h, int32_t epoch, const int64_t* order, w2v_dev_stats* stats);
/* The same, enqueued on the handle's stream; `order_dev` is a device array or NULL. */
int w2v_dev_train_epoch_async(w2v_dev* h, int32_t epoch, const int64_t* order_dev);
/* (w2v_dev_train_epoch returns W2V_ERR_DIVERGED, after the epoch, when any
 * sigma argument was non-finite; the model is then left as trained.) */
/* Train the `count` sentences listed in the device array `order_dev` (an
 * arbitrary slice of an epoch's order), enqueued on the handle's stream: lets a
 * caller cut an epoch into rounds between model-averaging points. */
int w2v_dev_train_sentences_async(w2v_dev* h, int32_t epoch, const int64_t* order_dev, int64_t count);
/* An epoch's sentence order (host array, n <= n_sentences ids) kept on the
 * device, and a slice [first, first + count) of it trained, enqueued on the
 * handle's stream: how a host loop cuts an epoch into rounds between
 * averaging points without device pointers. set_order waits for the work
 * already enqueued (it may still read the previous order). */
int w2v_dev_set_order(w2v_dev* h, const int64_t* order, int64_t n);
int w2v_dev_train_slice_async(w2v_dev* h, int32_t epoch, int64_t first, int64_t count);
int w2v_dev_synchronize(w2v_dev* h);
int w2v_dev_read_stats(w2v_dev* h, w2v_dev_stats* stats); /* cumulative; synchronizes */
int w2v_dev_reset_stats(w2v_dev* h);

/* Update policy of the parallel schedule (Hogwild across wavefronts; the
 * reference's OpenMP threads, Word2Vec.cpp:375-394, race the same way at a far
 * smaller scale). Three row classes, by frequency rank (the vocab is sorted by
 * count, Word2Vec.cpp:152):
 *  - private rows: the n hottest rows of the output layer (the NS target
 *    matrix — C for skip-gram, W for CBOW — or the n internal Huffman nodes
 *    nearest the root for HS). Each workgroup (up to 16 wavefronts) keeps its
 *    pending deltas for them in LDS (ds_add_f32); reads see the HBM value plus
 *    that delta. Every `flush_centers` centers of the workgroup the deltas go
 *    to HBM with float atomics, scaled so that a row which k workgroups update
 *    in one interval moves by at most average_over/k of their sum (local SGD
 *    on the rows every wavefront touches; without it ~10^4 concurrent stale
 *    updates of those rows diverge). -1 = as many as fit, at most 64 (default);
 *    0 = off;
 *  - hot rows: rows of W and C with index < hot_rows, and the hot_rows internal
 *    Huffman nodes nearest the root, take memory-side float atomic adds: no
 *    update is lost however many wavefronts hit the row. W2V_HOT_AUTO (-2,
 *    the default) = chosen per launch from the corpus statistics: the rows
 *    and nodes whose expected updates in flight (wavefronts x expected
 *    updates per center) reach the thresholds of w2v_dev_set_hot_auto
 *    (W / C rows: 1 by default — round 3's 2 for large vocabularies cost
 *    configs[2] a similarity point against the sequential reference;
 *    nodes: 1);
 *    -1 = every row, 0 = none,
 *    k > 0 = the k most frequent;
 *  - the rest: plain read-modify-write (an update racing another on the same
 *    row can be lost, as between the reference's threads).
 * Same fp32 rounding per update in every class. None of this applies to the
 * sequential schedule (W2V_SCHED_SEQUENTIAL), which is reference-exact. */
#define W2V_HOT_AUTO (-2)
int w2v_dev_set_hot_rows(w2v_dev* h, int64_t hot_rows);
/* Thresholds of the automatic hot rows: expected updates of a W / C row, of
 * a Huffman node, in flight across the chip (rows >= 0, 0 = the default, 1;
 * nodes > 0, default 1). */
int w2v_dev_set_hot_auto(w2v_dev* h, float tau_rows, float tau_nodes);
/* The thresholds the last parallel launch used (additive). */
int w2v_dev_hot_tau(w2v_dev* h, float* tau_rows, float* tau_nodes);
/* The update policy the last parallel launch used: hot W / C rows, hot
 * Huffman nodes, LDS-private output rows, LDS-private context rows. */
int w2v_dev_policy(w2v_dev* h, int64_t* hot_rows, int64_t* hot_nodes, int32_t* private_rows, int32_t* context_rows);
/* The flush intervals (workgroup centers) of the LDS-private output and
 * context rows the last parallel launch used (0 = that range was empty).
 * Auto for HS: the fewest of 64 ... 1024 that still gives every workgroup
 * >= 32 flushes per launch (context rows at half); NS: 1024. Additive; no
 * reference counterpart. */
int w2v_dev_flush_policy(w2v_dev* h, int32_t* flush_centers, int32_t* context_flush);
/* Expected updates per raw corpus token of every row of matrix `which` (0 W,
 * 1 C, 2 synapses1; n = its row count), from the uploaded vocab and corpus
 * statistics: what the flush scales, the hot-row threshold and the replica
 * exchange's per-row divisors are computed from. Additive. */
int w2v_dev_row_update_rates(w2v_dev* h, int32_t which, double* out, int64_t n);
/* LDS-private output rows per workgroup (-1, the default = automatic: as
 * many as fit the LDS budget, at most 64 for CBOW and HS, 96 for skip-gram NS,
 * 128 for skip-gram NS on a vocabulary >= 500 K words (rows past the 64th
 * flush with a gentler average), 96 Huffman nodes for CBOW-HS on a vocabulary
 * >= 50 K words when 63 context rows still fit (nodes 64..95 flushed at up to
 * 4 averaged contributions), 128 nodes for skip-gram HS (all at up to 4);
 * DESIGN.md §4.1). n > 0 asks for up to 128;
 * 0 disables them. Additive; no reference counterpart. */
int w2v_dev_set_private_rows(w2v_dev* h, int32_t n);
/* With private_rows = -1: privatise only the rows (Huffman nodes for HS, and
 * CBOW context rows) a center updates at least `mu` times on average, from
 * the corpus statistics (0 = no rate limit: as many as fit, up to the
 * automatic count of w2v_dev_set_private_rows; -1, the
 * default = 0.1 for a launch with fewer sentences than the chip holds waves,
 * else no limit). */
int w2v_dev_set_private_rate(w2v_dev* h, float mu);
/* The rate limit the last parallel launch used (0 = none). Additive. */
int w2v_dev_private_rate_used(w2v_dev* h, float* mu);
/* The waves-in-flight cap the last parallel per-pair launch chose for itself
 * (0: none, or the caller's w2v_dev_set_max_waves). With max_waves 0 a
 * launch keeps waves x (rows a kept center updates) / V <= 64: past that the
 * Hogwild staleness of an average row feeds on itself (a 1.8 K-word vocab at
 * window 150 / negative 80 diverges from 128 waves up, as the reference's own
 * OpenMP loop does on 8 threads). Every benchmarked shape stays uncapped. */
int w2v_dev_wave_cap_used(w2v_dev* h, int64_t* waves);
/* 1 if the last launch ran the low-occupancy deep-pipeline HS kernel (the
 * large-vocabulary HS policy's capped launches; environment W2V_DEEP_HS=1
 * forces it for any HS launch without negatives, 0 disables it). */
int w2v_dev_deep_used(w2v_dev* h, int32_t* deep);
/* The replica count the update policy assumes (no reference counterpart: the
 * reference trains one model). w2v_group_create sets it to the group's ranks;
 * the one-GPU rehearsal of an N-rank run (each rank a one-rank group, the
 * ranks combined over gloo) sets it to N, so its launches use the policy an
 * N-GPU run uses (shared negatives: no private C rows in a replica group).
 * n >= 1. */
int w2v_dev_set_replica_count(w2v_dev* h, int32_t n);
int w2v_dev_replica_count(w2v_dev* h, int32_t* n);
/* flush_centers: workgroup centers between flushes (0 = auto: 1024 for NS, 64
 * for HS); average_over: the concurrency a private row's summed deltas are
 * scaled down to (default 8; 0 = plain sum). */
int w2v_dev_set_private_sync(w2v_dev* h, int32_t flush_centers, float average_over);
/* CBOW only: privatise the `rows` hottest context rows of C (a window's
 * contexts are not subsampled, Word2Vec.cpp:286-300, so the most frequent
 * words sit in most windows) in LDS as well, beside the output rows, flushed
 * every flush_centers workgroup centers, scaled to at most 8 (CBOW-HS, the
 * output rows' average) or 128 (CBOW-NS) concurrent contributions. rows: -1 =
 * auto (as many as fit beside the output rows, at most 64);
 * 0 = off (those rows then take the hot-row atomics). flush_centers: 0 =
 * auto (HS: half the output rows' interval; NS: 256). */
int w2v_dev_set_context_private(w2v_dev* h, int32_t rows, int32_t flush_centers);
/* Cap on wavefronts in flight in the parallel schedule (0 = as many as fit,
 * the default). Fewer wavefronts, less staleness, less throughput. */
int w2v_dev_set_max_waves(w2v_dev* h, int64_t n);

/* Update formulation of the training kernels. W2V_UPDATE_PER_PAIR (default)
 * is the reference's train_sentence_sg/cbow (Word2Vec.cpp:273-353).
 * W2V_UPDATE_SHARED_NEGATIVES is the minibatch skip-gram of BASELINE
 * configs[4], a new formulation with no reference counterpart (restated in
 * oracle/w2v_oracle.cpp:sgsn_sentence): per kept center, the unique context
 * ids of its (shrunk) window are the inputs (W rows, weighted by multiplicity),
 * the center plus `negative` draws shared by the whole window the outputs (C
 * rows), and the window's updates are the three GEMMs L = W_in C_out^T,
 * dW_in = E C_out, dC_out = E^T W_in on the matrix cores. Skip-gram NS only,
 * negative <= 15, window <= 8, Philox draws, row pitch 64 * {1..8,10,12,14,16}
 * floats (W2V_ERR_UNSUPPORTED otherwise). Its parallel-schedule policy:
 * rows below hot_rows add their deltas with memory-side atomics, frequent
 * rows are read and written device-coherently, and private_rows (auto: <= 4)
 * of the hottest C rows are privatised per workgroup, flushed every
 * flush_centers (auto: 1024) centers. */
int w2v_dev_set_update(w2v_dev* h, int32_t mode);

/* Word2Vec::train_sentence_* take alpha from the caller (Word2Vec.h:83-84):
 * alpha > 0 makes every following epoch use it instead of the schedule of
 * Word2Vec.cpp:379-380; alpha <= 0 restores the schedule. */
int w2v_dev_set_fixed_alpha(w2v_dev* h, float alpha);

/* Replaces: negative_sampling / hierarchical_softmax called on their own
 * (Word2Vec.cpp:232-271, public API Word2Vec.h:81-82). Applies, in order, the
 * n target updates to `rows` (host, n dense rows of word_dim floats, read and
 * written; the rows must be distinct — they are the unique NS targets or the
 * nodes of one Huffman path) with codes[t] (HS: Huffman code; NS: 1 - label),
 * input `x` and gradient accumulator `grad` (host, word_dim floats, read and
 * written). hs_form selects the HS arithmetic (g = (1 - code - f) * alpha in
 * double, :241-242) or the NS one (g = (label - f) * alpha, :263-264). */
int w2v_dev_apply_rows(w2v_dev* h, float* rows, const uint8_t* codes, int32_t n, const float* x,
                       float* grad, float alpha, int32_t hs_form);

/* ---------------------------------------------------------------------------
 * Multi-GPU data parallelism (BASELINE configs[3], configs[4] at 2/4/8 GPUs;
 * new: the reference has only OpenMP threads on one model, Word2Vec.cpp:375-394).
 * Every replica (a w2v_dev handle with its model resident; all replicas start
 * from the same weights) trains its shard of the sentences;
 * w2v_group_average_async exchanges what the replicas learned since the last
 * exchange, ordered on each replica's stream after the work enqueued so far:
 * D_i = M_i - P, A = sum_i D_i (one ncclAllReduce per matrix over xGMI),
 * M_i = P + A / c per row: W2V_GROUP_SUM (default) c = 1 (every update
 * counts once, as in the reference's one shared model);
 * W2V_GROUP_ROW_AVERAGE c = the number of replicas that changed the row;
 * W2V_GROUP_AVERAGE c = R (model averaging: the mean of the replicas). One
 * process may drive several replicas (one per device: ncclCommInitAll), or
 * each process one or more with ranks from a shared unique id (one process
 * per GPU: rank 0 calls w2v_group_unique_id and hands the bytes to the others
 * out of band). Replicas on ONE device in one process are averaged by a
 * kernel instead (RCCL cannot put two ranks on one GPU).
 * Overlap (w2v_group_set_overlap(g, 1)): the all-reduce runs on a
 * communication stream while the next slice trains, and is folded in at the
 * next call (M += A / c - D: the other replicas' updates): the exchange is
 * delayed by one round, hidden behind compute. w2v_group_finish folds in the
 * last pending exchange and synchronises. The caller keeps the alpha schedule
 * global (w2v_dev_set_progress_async, w2v_dev_set_train_words).
 * ------------------------------------------------------------------------- */
#define W2V_GROUP_ID_BYTES 128
typedef struct w2v_group w2v_group;
int w2v_group_unique_id(uint8_t* id /* W2V_GROUP_ID_BYTES */);
/* members: the n handles this process drives (same model shape). unique_id
 * NULL: all replicas are in this process (nranks = n). Otherwise this
 * process's replicas are ranks [first_rank, first_rank + n) of nranks; with a
 * unique id even nranks = 1 builds the RCCL communicator and runs every
 * round's delta -> ncclAllReduce -> fold (the model is unchanged by it: the
 * sum of one replica's deltas), so one GPU exercises the exchange path. Each
 * member learns the group's replica count (nranks), which its update policy
 * reads from then on: with more than one replica, shared-negatives launches
 * above negative 5 keep no LDS-private rows. */
int w2v_group_create(w2v_dev** members, int32_t n, const uint8_t* unique_id, int32_t nranks, int32_t first_rank,
                     w2v_group** out);
void w2v_group_destroy(w2v_group* g);
int w2v_group_set_overlap(w2v_group* g, int32_t on);
#define W2V_GROUP_SUM 0
#define W2V_GROUP_AVERAGE 1
#define W2V_GROUP_ROW_AVERAGE 2
#define W2V_GROUP_ADAPTIVE 3 /* per row: the sum divided by max(1, |sum D|^2 / sum |D|^2) */
#define W2V_GROUP_SPLIT 4    /* per row: the mean for rows saturated within a round, else the sum */
#define W2V_GROUP_SATURATION 5 /* per row: the sum divided by a smooth function of the row's updates per round */
int w2v_group_set_mode(w2v_group* g, int32_t mode);
/* W2V_GROUP_SPLIT: rows a replica is expected to update >= saturated_updates
 * times in a round of tokens_per_round raw tokens (the corpus statistics of
 * member 0) take the mean of the replicas' updates, the rest their sum
 * (saturated_updates 0: every row the mean). */
int w2v_group_set_split(w2v_group* g, int64_t tokens_per_round, float saturated_updates);
/* W2V_GROUP_SATURATION: the sum divided per row by
 * c = R (1 - (1 - beta)^u) / (1 - (1 - beta)^(R u)), u = the row's expected
 * updates per replica in a round of tokens_per_round raw tokens (member 0's
 * corpus statistics) and beta the contraction of one update: what one model
 * updating the row R u times in a row would move it (the sum for rarely
 * updated rows, the mean for rows every replica saturates within the round). */
int w2v_group_set_saturation(w2v_group* g, int64_t tokens_per_round, float beta);
int w2v_group_split_rows(w2v_group* g, int64_t* rows); /* rows with a divisor > 1 (all matrices) */
/* The per-row divisors W2V_GROUP_SPLIT / SATURATION apply to matrix `which`
 * (n = its row count; all 1 in the other modes). */
int w2v_group_row_divisors(w2v_group* g, int32_t which, float* out, int64_t n);
int w2v_group_average_async(w2v_group* g);
/* The same exchange over the hottest rows only: rows [0, rows) of W and C
 * (the most frequent words) and the `rows` Huffman nodes nearest the root of
 * synapses1 (rows == 0: all). The other rows keep their own updates until a
 * later exchange covers them (their deltas stay relative to the last exchange
 * that did), so frequent hot-row exchanges between full ones are exact. */
int w2v_group_average_rows_async(w2v_group* g, int64_t rows);
int w2v_group_finish(w2v_group* g);
int w2v_group_info(w2v_group* g, int32_t* nranks, int32_t* local, int32_t* overlap, int64_t* rounds);

#ifdef __cplusplus
}
#endif
#endif /* W2V_DEV_H */
