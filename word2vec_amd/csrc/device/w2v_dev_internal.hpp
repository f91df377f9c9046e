// w2v_dev_internal.hpp — what the C-ABI's translation units share (not part of
// the public boundary, include/w2v_dev.h).
#pragma once
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdint>
#include <string>
#include <vector>

#include "w2v_dev.h"
#include "w2v_ingest.h"

namespace w2v {

// Record `msg` as this thread's w2v_dev_last_error(); returns `code`.
int set_error(int code, const std::string& msg);

struct DevInfo {
  int device;
  hipStream_t stream;
  int64_t V;
};
DevInfo dev_info(const w2v_dev* h);
// The replicas of the exchange group a handle joined (w2v_group_create: all
// ranks' members; 1 = none). The update policy reads it (launch_train). It
// stays after the group is destroyed (the group may outlive no handle, but a
// handle may outlive its group; it then keeps the replicas' policy).
void set_replicas(w2v_dev* h, int32_t n);

// Expected updates of each row of matrix k (0 = W, 1 = C, 2 = synapses1) per
// corpus token, from the corpus statistics the handle holds (the rates the
// update policy uses); false when the statistics are missing.
bool row_update_rates(w2v_dev* h, int k, std::vector<double>& out);

// The device samples of a mapped ingest (w2v_ingest.hip) for w2v_dev_adopt_corpus.
struct IngestView {
  bool ok;
  int device;
  const int32_t* ids;
  int64_t n_ids;
  const int64_t* offsets;  // n_sentences + 1
  int64_t n_sentences;
  int64_t train_words;
  const int64_t* hist;  // host: tokens per vocab id, n_vocab entries
  int64_t n_vocab;
};
IngestView ingest_view(const w2v_ingest* g);

// roctx range for the duration of a scope (rocprofv3 --marker-trace shows the
// C-ABI's uploads, epochs and replica exchanges on the timeline).
struct Range {
  explicit Range(const char* name) { roctxRangePushA(name); }
  ~Range() { roctxRangePop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

}  // namespace w2v
