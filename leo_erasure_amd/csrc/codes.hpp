// codes.hpp — GF(2^w) fields and the coding matrices of the four leo_erasure
// classes, as the engine's host side builds them before launching GPU work.
//
// Reference call sites whose matrices these reproduce:
//   vandrs      reed_sol_vandermonde_coding_matrix   c_src/rscoding.cpp:67,143,194
//   cauchyrs    cauchy_good_general_coding_matrix +  c_src/cauchycoding.cpp:38-39,147-148,197-198
//               jerasure_matrix_to_bitmatrix
//   liberation  liberation_coding_bitmatrix          c_src/liberationcoding.cpp:39,146,194
//   isars       gf_gen_cauchy1_matrix                c_src/irscoding.cpp:68,131,173
// and the decoding maps of jerasure_matrix_decode_data / _selected,
// jerasure_schedule_decode_*_lazy and IRSCoding::gf_gen_decode_matrix.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace leoec {

// GF(2^w) with gf-complete's default primitive polynomial for w.
class Field {
 public:
  explicit Field(int w);
  int w() const { return w_; }
  uint32_t mul(uint32_t a, uint32_t b) const;
  uint32_t inv(uint32_t a) const;
  uint32_t div(uint32_t a, uint32_t b) const { return b ? mul(a, inv(b)) : 0xFFFFFFFFu; }
  // number of ones in the w x w GF(2) matrix of "multiply by a"
  int bit_weight(uint32_t a) const;

 private:
  uint32_t slow_mul(uint32_t a, uint32_t b) const;
  int w_;
  uint64_t poly_;                  // including x^w
  std::vector<uint32_t> log_, exp_;  // w <= 16
};

const Field& field(int w);  // process-wide, built once per w

// Dense GF matrix, row-major.
struct GfMatrix {
  int rows = 0, cols = 0;
  std::vector<uint32_t> a;
  uint32_t& at(int r, int c) { return a[(size_t)r * cols + c]; }
  uint32_t at(int r, int c) const { return a[(size_t)r * cols + c]; }
};

// GF(2) matrix with rows packed in 64-bit words.
struct BitMatrix {
  int rows = 0, cols = 0, words = 0;
  std::vector<uint64_t> bits;
  void resize(int r, int c) {
    rows = r; cols = c; words = (c + 63) / 64;
    bits.assign((size_t)r * words, 0);
  }
  bool get(int r, int c) const { return (bits[(size_t)r * words + c / 64] >> (c % 64)) & 1; }
  void set(int r, int c, bool v) {
    uint64_t& x = bits[(size_t)r * words + c / 64];
    x = v ? (x | (1ull << (c % 64))) : (x & ~(1ull << (c % 64)));
  }
  uint64_t* row(int r) { return &bits[(size_t)r * words]; }
  const uint64_t* row(int r) const { return &bits[(size_t)r * words]; }
};

// status-returning builders (0 = ok, <0 = leoec_status)
int vandermonde_coding_matrix(int k, int m, int w, GfMatrix* out);
int cauchy_good_coding_matrix(int k, int m, int w, GfMatrix* out);
int isal_cauchy1_coding_matrix(int k, int m, GfMatrix* out);  // rows k..k+m-1 only
int liberation_coding_bitmatrix(int k, int w, BitMatrix* out);
void expand_to_bitmatrix(const GfMatrix& m, int w, BitMatrix* out);

int gf_invert(const GfMatrix& in, int w, GfMatrix* out);  // -11 if singular
int bit_invert(const BitMatrix& in, BitMatrix* out);      // -11 if singular

}  // namespace leoec
