// w2v_corpus.h — streaming corpus ingestion (corpus.cpp): mapped files,
// threaded tokenisation, the reference's vocabulary and samples without
// vector<vector<string>>. Internal to libword2vec_amd (used by Word2Vec's
// build_vocab_file / train_file).
#ifndef W2V_AMD_CORPUS_H
#define W2V_AMD_CORPUS_H

#include <cstddef>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace w2v_corpus {

enum Format {
  kLines,  // one sentence per line (line_docs, Word2Vec.cpp:19-30)
  kText8   // whitespace tokens in 1000-token sentences (main.cpp:63-92)
};
Format parse_format(const std::string& f);

class File {  // read-only mapping of a whole file
 public:
  explicit File(const std::string& path);
  ~File();
  File(const File&) = delete;
  File& operator=(const File&) = delete;
  const char* data() const { return data_; }
  size_t size() const { return size_; }

 private:
  int fd_ = -1;
  const char* data_ = nullptr;
  size_t size_ = 0;
};

struct Counts {
  std::vector<std::pair<std::string, int64_t>> words;  // distinct words, in order of first occurrence
  int64_t raw_tokens = 0;
};
// Word counts of the corpus (threads <= 0: all hardware threads).
Counts count_words(const File& f, Format fmt, int threads);

struct Samples {
  std::vector<int32_t> ids;      // in-vocab tokens (build_sample), sentence by sentence
  std::vector<int64_t> offsets;  // sentence s = ids[offsets[s], offsets[s+1])
  int64_t raw_tokens = 0;        // train_words (Word2Vec.cpp:362-363)
};
// build_sample over the file with `index` (word -> vocab index).
Samples samples(const File& f, Format fmt, int threads, const std::unordered_map<std::string, int32_t>& index);

}  // namespace w2v_corpus

#endif  // W2V_AMD_CORPUS_H
