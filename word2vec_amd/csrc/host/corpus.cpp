// corpus.cpp — streaming corpus ingestion for files too large for the
// reference's vector<vector<string>>: the file is mapped,
// tokenised by host threads over byte ranges, and turned into
//   * the reference's vocabulary, bit-exact: Word2Vec::build_vocab
//     (Word2Vec.cpp:132-169) counts in an unordered_map<string,int> whose
//     iteration order depends only on the order in which distinct words are
//     first inserted; here the threads count in private tables, and the merged
//     words are inserted into that same map type in order of first occurrence;
//   * build_sample's token lists (Word2Vec.cpp:212-230) as int32 ids plus
//     sentence offsets, and train()'s train_words (raw tokens, :362-363).
// Sentences are either lines (line_docs, Word2Vec.cpp:19-30: getline, then
// whitespace tokens; empty lines are empty sentences) or the reference CLI's
// text8 reader (main.cpp:63-92: whitespace tokens in 1000-token sentences).
// Tokens split on the C-locale isspace set, as operator>> does.
#include "w2v_corpus.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <utility>

namespace w2v_corpus {
namespace {

struct SpaceTable {  // the C-locale isspace set, as a byte lookup
  bool t[256];
  SpaceTable() {
    for (int i = 0; i < 256; ++i) t[i] = false;
    const char* sp = " \t\n\v\f\r";
    for (const char* c = sp; *c; ++c) t[(unsigned char)*c] = true;
  }
};
const SpaceTable kSpace;
inline bool is_space(char c) { return kSpace.t[(unsigned char)c]; }

inline uint64_t hash_bytes(const char* p, size_t n) {  // FNV-1a, 64-bit
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ (unsigned char)p[i]) * 1099511628211ull;
  return h;
}

// Open-addressing table of words that live in the mapped file (no copies).
// A slot keeps the word's first 16 bytes, so matching a word of <= 16 bytes
// (nearly all of them) touches the slot only, not its first occurrence in the
// file (a random access into a file far larger than the caches).
struct WordTable {
  static const uint32_t kHead = 16;
  struct Slot {
    uint64_t hash = 0;
    char head[kHead];
    size_t off = 0;     // first occurrence (byte offset in the file)
    uint32_t len = 0;   // 0 = empty slot
    int32_t id = -1;
    int64_t count = 0;
  };
  std::vector<Slot> slots;
  size_t used = 0;
  const char* base = nullptr;

  explicit WordTable(const char* b, size_t cap = 1 << 16) : slots(cap), base(b) {}

  Slot* find_or_insert(const char* p, uint32_t n, uint64_t h, bool insert) {
    if (insert && (used + 1) * 2 > slots.size()) grow();
    size_t m = slots.size() - 1, i = (size_t)h & m;
    for (;;) {
      Slot& s = slots[i];
      if (s.len == 0) {
        if (!insert) return nullptr;
        s.hash = h;
        s.off = (size_t)(p - base);
        s.len = n;
        std::memcpy(s.head, p, n < kHead ? n : kHead);
        ++used;
        return &s;
      }
      if (s.hash == h && s.len == n && same(s, p, n)) return &s;
      i = (i + 1) & m;
    }
  }

  bool same(const Slot& s, const char* p, uint32_t n) const {
    const uint32_t k = n < kHead ? n : kHead;
    if (std::memcmp(s.head, p, k) != 0) return false;
    return n <= kHead || std::memcmp(base + s.off + kHead, p + kHead, n - kHead) == 0;
  }

  void grow() {
    std::vector<Slot> old;
    old.swap(slots);
    slots.assign(old.size() * 2, Slot());
    size_t m = slots.size() - 1;
    for (const Slot& s : old)
      if (s.len) {
        size_t i = (size_t)s.hash & m;
        while (slots[i].len) i = (i + 1) & m;
        slots[i] = s;
      }
  }
};

// Visit the tokens of [b, e): fn(token pointer, length); at every '\n' (lines
// format only) call line().
template <class F, class L>
void scan(const char* base, size_t b, size_t e, F fn, L line) {
  size_t i = b;
  while (i < e) {
    const char c = base[i];
    if (is_space(c)) {
      if (c == '\n') line();
      ++i;
      continue;
    }
    size_t j = i;
    while (j < e && !is_space(base[j])) ++j;
    fn(base + i, j - i);
    i = j;
  }
}

}  // namespace

File::File(const std::string& path) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) throw std::runtime_error("w2v_corpus: cannot open " + path);
  struct stat st;
  if (::fstat(fd_, &st) != 0) throw std::runtime_error("w2v_corpus: cannot stat " + path);
  size_ = (size_t)st.st_size;
  if (size_ > 0) {
    void* p = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (p == MAP_FAILED) throw std::runtime_error("w2v_corpus: cannot map " + path);
    ::madvise(p, size_, MADV_SEQUENTIAL);
    data_ = static_cast<const char*>(p);
  }
}

File::~File() {
  if (data_) ::munmap(const_cast<char*>(data_), size_);
  if (fd_ >= 0) ::close(fd_);
}

Format parse_format(const std::string& f) {
  if (f == "lines") return kLines;
  if (f == "text8") return kText8;
  throw std::runtime_error("w2v_corpus: format must be \"lines\" or \"text8\", not \"" + f + "\"");
}

// Byte ranges for the threads, cut after a '\n' (lines) or a whitespace byte
// (text8) so that no token or line spans two ranges.
std::vector<std::pair<size_t, size_t>> split(const File& f, Format fmt, int threads) {
  const size_t n = f.size();
  const char* p = f.data();
  int t = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
  t = (int)std::min<size_t>((size_t)t, std::max<size_t>(1, n / (1 << 20)));  // >= 1 MiB per range
  std::vector<std::pair<size_t, size_t>> r;
  size_t b = 0;
  for (int k = 1; k <= t; ++k) {
    size_t e = (k == t) ? n : n / (size_t)t * (size_t)k;
    if (e < b) e = b;
    while (e < n && !(fmt == kLines ? p[e - 1] == '\n' : is_space(p[e - 1]))) ++e;
    r.emplace_back(b, e);
    b = e;
  }
  return r;
}

template <class Fn>
static void parallel(size_t n, Fn fn) {
  std::vector<std::thread> th;
  for (size_t k = 1; k < n; ++k) th.emplace_back(fn, k);
  fn(0);
  for (auto& x : th) x.join();
}

Counts count_words(const File& f, Format fmt, int threads) {
  const auto ranges = split(f, fmt, threads);
  std::vector<WordTable> tabs(ranges.size(), WordTable(f.data()));
  std::vector<int64_t> toks(ranges.size(), 0);
  parallel(ranges.size(), [&](size_t k) {
    WordTable& t = tabs[k];
    int64_t nt = 0;
    scan(f.data(), ranges[k].first, ranges[k].second,
         [&](const char* w, size_t n) {
           t.find_or_insert(w, (uint32_t)n, hash_bytes(w, n), true)->count += 1;
           ++nt;
         },
         [] {});
    toks[k] = nt;
  });
  // merge in range order: the first occurrence of a word is its smallest offset
  WordTable all(f.data(), 1 << 20);
  for (auto& t : tabs)
    for (const auto& s : t.slots)
      if (s.len) {
        auto* g = all.find_or_insert(f.data() + s.off, s.len, s.hash, true);
        g->count += s.count;
        g->off = std::min(g->off, s.off);
      }
  std::vector<const WordTable::Slot*> order;
  order.reserve(all.used);
  for (const auto& s : all.slots)
    if (s.len) order.push_back(&s);
  std::sort(order.begin(), order.end(),
            [](const WordTable::Slot* a, const WordTable::Slot* b) { return a->off < b->off; });
  Counts c;
  for (auto t : toks) c.raw_tokens += t;
  c.words.reserve(order.size());
  for (auto* s : order) c.words.emplace_back(std::string(f.data() + s->off, s->len), s->count);
  return c;
}

Samples samples(const File& f, Format fmt, int threads, const std::unordered_map<std::string, int32_t>& index) {
  const auto ranges = split(f, fmt, threads);
  // read-only lookup table of the vocabulary, keyed by the words' bytes
  std::vector<std::string> keys;
  keys.reserve(index.size());
  std::string arena;
  std::vector<std::pair<size_t, int32_t>> where;
  for (const auto& kv : index) {
    where.emplace_back(arena.size(), kv.second);
    arena += kv.first;
  }
  WordTable vt(arena.data(), 1 << 16);
  {
    size_t k = 0;
    for (const auto& kv : index) {
      const char* p = arena.data() + where[k].first;
      vt.find_or_insert(p, (uint32_t)kv.first.size(), hash_bytes(p, kv.first.size()), true)->id = where[k].second;
      ++k;
    }
  }
  struct Part {
    std::vector<int32_t> ids;
    std::vector<int64_t> lens;      // lines: kept tokens per line started in this range
    std::vector<int64_t> raw_at;    // text8: raw token index of each kept id (for the 1000-token cut)
    int64_t raw = 0;
    bool open_line = false;          // lines: a line is still open at the end of the range
  };
  std::vector<Part> parts(ranges.size());
  parallel(ranges.size(), [&](size_t k) {
    Part& pt = parts[k];
    int64_t cur = 0;
    bool open = false;
    scan(f.data(), ranges[k].first, ranges[k].second,
         [&](const char* w, size_t n) {
           const auto* s = vt.find_or_insert(w, (uint32_t)n, hash_bytes(w, n), false);
           if (s) {
             pt.ids.push_back(s->id);
             if (fmt == kText8) pt.raw_at.push_back(pt.raw);
             ++cur;
           }
           ++pt.raw;
           open = true;
         },
         [&] {
           if (fmt == kLines) pt.lens.push_back(cur);
           cur = 0;
           open = false;
         });
    // a range ends after '\n' unless it is the file's last: its tail is a line
    // only if it holds bytes (getline returns a final unterminated line)
    if (fmt == kLines && ranges[k].second > ranges[k].first &&
        f.data()[ranges[k].second - 1] != '\n') {
      pt.lens.push_back(cur);
    }
    (void)open;
  });
  Samples out;
  size_t total = 0;
  for (auto& p : parts) total += p.ids.size();
  out.ids.reserve(total);
  out.offsets.assign(1, 0);
  if (fmt == kLines) {
    for (auto& p : parts) {
      for (int64_t n : p.lens) out.offsets.push_back(out.offsets.back() + n);
      out.ids.insert(out.ids.end(), p.ids.begin(), p.ids.end());
      out.raw_tokens += p.raw;
    }
  } else {
    const int64_t kSentence = 1000;  // main.cpp:66
    int64_t raw0 = 0;
    for (auto& p : parts) out.raw_tokens += p.raw;
    const int64_t n_sent = (out.raw_tokens + kSentence - 1) / kSentence;
    std::vector<int64_t> per((size_t)n_sent, 0);
    for (auto& p : parts) {
      for (int64_t r : p.raw_at) per[(size_t)((raw0 + r) / kSentence)] += 1;
      out.ids.insert(out.ids.end(), p.ids.begin(), p.ids.end());
      raw0 += p.raw;
    }
    for (int64_t n : per) out.offsets.push_back(out.offsets.back() + n);
  }
  return out;
}

}  // namespace w2v_corpus
