/*
 * w2v_host.h — C-ABI of the host-side products that feed the device hot path
 * (libword2vec_amd.so). Each function restates one reference step exactly
 * (same float arithmetic, same libstdc++ heap tie-breaking), so the products
 * are bit-identical to what Word2Vec::build_vocab computes:
 *
 *   w2v_host_sample_probs   precalc_sampling     Word2Vec.cpp:115-130
 *   w2v_host_table_bounds   make_table           Word2Vec.cpp:81-113  (as V+1 boundaries)
 *   w2v_host_table_fill     make_table           Word2Vec.cpp:81-113  (expanded)
 *   w2v_host_huffman        create_huffman_tree  Word2Vec.cpp:32-79   (CSR codes/points)
 *
 * `counts` are in vocab index order (descending, as build_vocab sorts them).
 */
#ifndef W2V_HOST_H
#define W2V_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* w2v_host_version(void);

/* Word::sample_probability for every word. */
void w2v_host_sample_probs(const int64_t* counts, int64_t V, float subsample_threshold, float* out);

/* First index in the unigram table of every word; out[V] = table_size. Words
 * the reference's loop never reaches get empty ranges at the end. */
void w2v_host_table_bounds(const int64_t* counts, int64_t V, int32_t table_size, int64_t* out);

/* The expanded table (n = table_size entries) from the boundaries. */
void w2v_host_table_fill(const int64_t* bounds, int64_t V, uint32_t* table, int64_t n);

/* Huffman codes/points, CSR by word. Returns the total path length; writes
 * codes/points only if their capacity `cap` suffices (call with cap = 0 to
 * size). offsets has V+1 entries. Returns -1 on V < 2. */
int64_t w2v_host_huffman(const int64_t* counts, int64_t V, uint8_t* codes, int32_t* points,
                         int64_t* offsets, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* W2V_HOST_H */
