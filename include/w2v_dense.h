// w2v_dense.h — the small dense-row vocabulary the Word2Vec class API exposes.
//
// The reference types its public matrices and vectors with Eigen
// (RMatrixXf = Matrix<float, Dynamic, Dynamic, RowMajor>, RowVectorXf;
// Word2Vec.h:18,27,53,81-82). This framework keeps the model in HBM and only
// mirrors it on the host for the class API and the vector files, so it ships
// its own row-major fp32 types with the subset of that surface the class and
// its callers use (rows/cols/row/data/Zero/setZero/dot/+=/scalar ops and the
// IOFormat used by save_word2vec). It is not Eigen and does not try to be.
#ifndef W2V_DENSE_H
#define W2V_DENSE_H

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <ostream>
#include <vector>

namespace w2v_dense {

typedef std::ptrdiff_t Index;

enum { StreamPrecision = -1, FullPrecision = -2 };
enum { DontAlignCols = 1 };

// Formatting of a row as save_word2vec writes it (Word2Vec.cpp:400,434):
// coefficients separated by one space at the stream's precision.
struct IOFormat {
  int precision;
  int flags;
  explicit IOFormat(int p = StreamPrecision, int f = 0) : precision(p), flags(f) {}
};

class RowVectorXf;

// A view of one row of a matrix (or of a whole vector); writes go through.
class RowRef {
 public:
  RowRef(float* p, Index n) : p_(p), n_(n) {}
  Index size() const { return n_; }
  Index cols() const { return n_; }
  float* data() { return p_; }
  const float* data() const { return p_; }
  float& operator[](Index k) { return p_[k]; }
  float operator[](Index k) const { return p_[k]; }
  float& operator()(Index k) { return p_[k]; }
  float operator()(Index k) const { return p_[k]; }
  template <class V>
  float dot(const V& o) const {  // sequential fp32 sum
    float s = 0.0f;
    for (Index k = 0; k < n_; ++k) s += p_[k] * o.data()[k];
    return s;
  }
  template <class V>
  RowRef& operator+=(const V& o) {
    for (Index k = 0; k < n_; ++k) p_[k] += o.data()[k];
    return *this;
  }
  template <class V>
  RowRef& operator=(const V& o) {
    for (Index k = 0; k < n_; ++k) p_[k] = o.data()[k];
    return *this;
  }
  RowRef& operator=(const RowRef& o) {
    for (Index k = 0; k < n_; ++k) p_[k] = o.p_[k];
    return *this;
  }
  struct Formatted {
    const float* p;
    Index n;
  };
  Formatted format(const IOFormat&) const { return Formatted{p_, n_}; }

 private:
  float* p_;
  Index n_;
};

inline std::ostream& operator<<(std::ostream& os, const RowRef::Formatted& f) {
  for (Index k = 0; k < f.n; ++k) {
    if (k) os << ' ';
    os << f.p[k];
  }
  return os;
}

class RowVectorXf {
 public:
  RowVectorXf() {}
  explicit RowVectorXf(Index n) : v_((size_t)n, 0.0f) {}
  RowVectorXf(const RowRef& r) : v_(r.data(), r.data() + r.size()) {}
  static RowVectorXf Zero(Index n) { return RowVectorXf(n); }
  Index size() const { return (Index)v_.size(); }
  Index cols() const { return (Index)v_.size(); }
  Index rows() const { return 1; }
  float* data() { return v_.data(); }
  const float* data() const { return v_.data(); }
  float& operator[](Index k) { return v_[(size_t)k]; }
  float operator[](Index k) const { return v_[(size_t)k]; }
  float& operator()(Index k) { return v_[(size_t)k]; }
  float operator()(Index k) const { return v_[(size_t)k]; }
  void setZero() { std::fill(v_.begin(), v_.end(), 0.0f); }
  void resize(Index n) { v_.assign((size_t)n, 0.0f); }
  RowVectorXf& operator=(const RowRef& r) {
    v_.assign(r.data(), r.data() + r.size());
    return *this;
  }
  template <class V>
  float dot(const V& o) const {
    float s = 0.0f;
    for (size_t k = 0; k < v_.size(); ++k) s += v_[k] * o.data()[k];
    return s;
  }
  template <class V>
  RowVectorXf& operator+=(const V& o) {
    for (size_t k = 0; k < v_.size(); ++k) v_[k] += o.data()[k];
    return *this;
  }
  RowVectorXf& operator/=(float s) {
    for (float& x : v_) x /= s;
    return *this;
  }
  RowVectorXf& operator*=(float s) {
    for (float& x : v_) x *= s;
    return *this;
  }
  RowRef row(Index) { return RowRef(v_.data(), size()); }
  RowRef::Formatted format(const IOFormat&) const { return RowRef::Formatted{v_.data(), size()}; }

 private:
  std::vector<float> v_;
};

// Row-major fp32 matrix (the reference's RMatrixXf).
class RMatrixXf {
 public:
  typedef float Scalar;
  typedef w2v_dense::Index Index;
  RMatrixXf() : r_(0), c_(0) {}
  RMatrixXf(Index r, Index c) : r_(r), c_(c), v_((size_t)(r * c), 0.0f) {}
  static RMatrixXf Zero(Index r, Index c) { return RMatrixXf(r, c); }
  Index rows() const { return r_; }
  Index cols() const { return c_; }
  Index size() const { return r_ * c_; }
  float* data() { return v_.data(); }
  const float* data() const { return v_.data(); }
  RowRef row(Index i) { return RowRef(v_.data() + i * c_, c_); }
  RowRef row(Index i) const { return RowRef(const_cast<float*>(v_.data()) + i * c_, c_); }
  float& operator()(Index i, Index j) { return v_[(size_t)(i * c_ + j)]; }
  float operator()(Index i, Index j) const { return v_[(size_t)(i * c_ + j)]; }
  void resize(Index r, Index c) {
    r_ = r;
    c_ = c;
    v_.assign((size_t)(r * c), 0.0f);
  }
  void setZero() { std::fill(v_.begin(), v_.end(), 0.0f); }

 private:
  Index r_, c_;
  std::vector<float> v_;
};

}  // namespace w2v_dense

#endif  // W2V_DENSE_H
