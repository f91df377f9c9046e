/*
 * w2v_ingest.h — corpus ingestion on the GPU: the
 * vocabulary count and build_sample's id mapping of a large corpus file,
 * bit-exact with the host readers.
 *
 * Replaces the host passes behind Word2Vec::build_vocab (Word2Vec.cpp:132-160:
 * the unordered_map<string,int> count in corpus order) and build_sample
 * (:212-230: strings -> in-vocab ids) for files read like line_docs
 * (Word2Vec.cpp:19-30: one sentence per line) or the reference CLI's text8
 * reader (main.cpp:63-92: 1000-token sentences). The bytes (a mapped file)
 * cross PCIe in chunks; tokenising (the C-locale isspace set, as
 * operator>>), hashing and counting run in gfx950 kernels against a device
 * hash table. The words come back in order of first occurrence with their
 * counts: inserting them into the reference's map type in that order gives
 * the map build_vocab builds (its iteration order depends only on the
 * insertion order of the distinct words), so the host keeps the exact
 * reference tie order (std::sort over that map, Word2Vec.cpp:143-160). Every
 * token is matched by two independent 64-bit hashes and its length; a
 * mismatch (a hash collision between two different words) fails the call
 * (W2V_ERR_UNSUPPORTED) instead of merging them. The samples (int32 ids +
 * int64 sentence offsets) stay in HBM and can be handed to a training handle
 * without a host copy (w2v_dev_adopt_corpus).
 *
 * Same conventions as w2v_dev.h: plain pointers, an int status (W2V_OK ...),
 * w2v_dev_last_error() for the message, synchronous calls.
 */
#ifndef W2V_INGEST_H
#define W2V_INGEST_H

#include <stdint.h>

#include "w2v_dev.h"

#ifdef __cplusplus
extern "C" {
#endif

#define W2V_INGEST_LINES 0 /* one sentence per line (line_docs)               */
#define W2V_INGEST_TEXT8 1 /* 1000-token sentences over the whole file (text8) */

typedef struct w2v_ingest w2v_ingest;

/* device: HIP ordinal (-1 = current). chunk_bytes: bytes per host -> device
 * transfer (0 = 1 GiB). */
int w2v_ingest_create(int32_t device, int32_t format, int64_t chunk_bytes, w2v_ingest** out);
void w2v_ingest_destroy(w2v_ingest* g);

/* Largest file (bytes) kept in HBM between the passes; 0 = always stream
 * the chunks, < 0 = the default (64 GiB). Set before w2v_ingest_count. */
int w2v_ingest_set_resident(w2v_ingest* g, int64_t max_bytes);

/* Pass 1 (Word2Vec.cpp:134-141): count the words of data[0, n_bytes). */
int w2v_ingest_count(w2v_ingest* g, const char* data, int64_t n_bytes);
/* Distinct words, raw tokens (train_words, :362-363) and sentences of pass 1. */
int w2v_ingest_summary(w2v_ingest* g, int64_t* n_words, int64_t* raw_tokens, int64_t* n_sentences);
/* Per distinct word, in ascending order of first occurrence: the byte offset
 * of its first occurrence in data, its length in bytes, its count. */
int w2v_ingest_words(w2v_ingest* g, int64_t* first_offset, int32_t* length, int64_t* count);

/* Pass 2 (build_sample, :212-230): vocab_index[k] is the vocab index of the
 * k-th word of w2v_ingest_words (-1: not in the vocab, dropped). The same
 * bytes as pass 1: a file of up to 64 GiB (w2v_ingest_set_resident) stays in HBM after pass 1 and pass
 * 2 reads that copy (one PCIe crossing); larger files are streamed again. */
int w2v_ingest_map(w2v_ingest* g, const char* data, int64_t n_bytes, const int32_t* vocab_index, int64_t n_words);
/* In-vocab ids, sentences, and train_words of pass 2. */
int w2v_ingest_samples_size(w2v_ingest* g, int64_t* n_ids, int64_t* n_sentences, int64_t* train_words);
/* Copy the samples to the host: ids (n_ids int32), offsets (n_sentences + 1 int64). */
int w2v_ingest_download(w2v_ingest* g, int32_t* ids, int64_t* offsets);
/* Hand the samples to a training handle on the same device (replaces
 * w2v_dev_upload_corpus; no host round trip). The ingest object keeps its
 * copy until destroyed. */
int w2v_dev_adopt_corpus(w2v_dev* h, w2v_ingest* g);

#ifdef __cplusplus
}
#endif
#endif /* W2V_INGEST_H */
