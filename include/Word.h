// Word.h — a vocabulary entry that is also a Huffman-tree node; same members
// and constructor as the reference's Word (/root/reference/Word.h:11-29).
#ifndef W2V_AMD_WORD_H
#define W2V_AMD_WORD_H

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

class Word {
 public:
  size_t index = 0;
  size_t count = 0;
  float sample_probability = 1.0f;
  std::string text;
  Word* left = nullptr;
  Word* right = nullptr;

  std::vector<size_t> codes;   // Huffman code, root -> leaf (0 = left, 1 = right)
  std::vector<size_t> points;  // internal-node ids (rows of synapses1), root -> leaf

  Word() {}
  Word(size_t index_, size_t count_, std::string text_, Word* left_ = nullptr, Word* right_ = nullptr)
      : index(index_), count(count_), text(std::move(text_)), left(left_), right(right_) {}
  ~Word() {}
};

typedef std::shared_ptr<Word> WordP;

#endif  // W2V_AMD_WORD_H
