// A caller shaped like the reference's CLI driver (/root/reference/main.cpp:
// 94-204, its call sequence and its environment: Eigen::initParallel(),
// omp_set_num_threads, unqualified std names, the 13-argument constructor,
// build_vocab -> init_weights(vocab.size()) -> save_vocab -> train ->
// save_word2vec of W or C), written against the reference's API only and
// compiled against include/Word2Vec.h unmodified. It reads one sentence per
// line (line_docs, Word2Vec.cpp:19-30) instead of ./text8.
// usage: ref_caller <corpus> <vectors out> <vocab out> <model: sg|cbow> <method: ns|hs>
#include "Word2Vec.h"

int main(int argc, char** argv) {
  Eigen::initParallel();
  if (argc < 6) {
    cout << "usage: ref_caller corpus vectors vocab model method" << endl;
    return 1;
  }
  string model = argv[4], train_method = argv[5];
  int negative = train_method == "ns" ? 5 : 0;
  float init_alpha = 0.05f;  // the reference forces 0.05 (cbow_mean is always set, main.cpp:180-181)
  Word2Vec w2v(1, 5, 2, 100000, 32, negative, 1e-3f, init_alpha, 2.5e-6f, true, 2, train_method, model);
  omp_set_num_threads(2);
  vector<vector<string>> sentences = w2v.line_docs(argv[1]);
  w2v.build_vocab(sentences);
  w2v.init_weights(w2v.vocab.size());
  w2v.save_vocab(argv[3]);
  w2v.train(sentences);
  if (model == "cbow" && train_method == "hs")
    w2v.save_word2vec(argv[2], w2v.C);
  else
    w2v.save_word2vec(argv[2], w2v.W);
  cout << "trained " << w2v.vocab.size() << " words" << endl;
  return 0;
}
