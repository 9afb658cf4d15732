// TEST DRIVER (CPU) for leo_erasure_amd/csrc/gfs_core.hpp: the bitsliced
// GF(2^16) / GF(2^32) multiply-accumulate that gfs_apply runs on the GPU,
// compiled with g++ and driven from tests/test_gfs_core.py against the
// oracle's field arithmetic.  Not part of the product.
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "../leo_erasure_amd/csrc/gfs_core.hpp"

namespace {

// As gfs_apply: a lane's 64 bytes are 16 registers (w = 16: 32 words;
// w = 32: 16 words, the packed layout), transpose<16>, then mac<16> or
// mac_p32.
template <int W, int R>
void region(int K, const uint32_t* coef, const uint8_t* in, size_t bytes, uint8_t* out) {
  constexpr size_t G = 64;
  for (size_t g = 0; g + G <= bytes; g += G) {
    uint32_t acc[R][16] = {};
    for (int j = 0; j < K; ++j) {
      uint32_t pl[16];
      std::memcpy(pl, in + (size_t)j * bytes + g, sizeof pl);
      leoec::gfs::transpose<16>(pl);
      uint32_t c[R];
      for (int r = 0; r < R; ++r) c[r] = coef[r * K + j];
      if (W == 32) leoec::gfs::mac_p32<R>(pl, acc, c);
      else leoec::gfs::mac<16, R>(pl, acc, c);
    }
    for (int r = 0; r < R; ++r) {
      leoec::gfs::transpose<16>(acc[r]);
      std::memcpy(out + (size_t)r * bytes + g, acc[r], sizeof acc[r]);
    }
  }
}

// The unpacked w = 32 form (32 words per lane, transpose<32>, mac<32>).
template <int R>
void region32u(int K, const uint32_t* coef, const uint8_t* in, size_t bytes, uint8_t* out) {
  constexpr size_t G = 128;
  for (size_t g = 0; g + G <= bytes; g += G) {
    uint32_t acc[R][32] = {};
    for (int j = 0; j < K; ++j) {
      uint32_t pl[32];
      std::memcpy(pl, in + (size_t)j * bytes + g, sizeof pl);
      leoec::gfs::transpose<32>(pl);
      uint32_t c[R];
      for (int r = 0; r < R; ++r) c[r] = coef[r * K + j];
      leoec::gfs::mac<32, R>(pl, acc, c);
    }
    for (int r = 0; r < R; ++r) {
      leoec::gfs::transpose<32>(acc[r]);
      std::memcpy(out + (size_t)r * bytes + g, acc[r], sizeof acc[r]);
    }
  }
}

template <int W>
int region_w(int R, int K, const uint32_t* coef, const uint8_t* in, size_t bytes, uint8_t* out) {
  switch (R) {
    case 1: region<W, 1>(K, coef, in, bytes, out); return 0;
    case 2: region<W, 2>(K, coef, in, bytes, out); return 0;
    case 3: region<W, 3>(K, coef, in, bytes, out); return 0;
    case 4: region<W, 4>(K, coef, in, bytes, out); return 0;
  }
  return -1;
}

}  // namespace

// out[r] = XOR_j coef[r*K + j] * in[j] over GF(2^w), word-wise (little
// endian), for K input regions of `bytes` each (a multiple of 32*w/8).
extern "C" int gfs_region(int w, int R, int K, const uint32_t* coef, const uint8_t* in,
                          size_t bytes, uint8_t* out) {
  if (w == 32) return region_w<32>(R, K, coef, in, bytes, out);
  if (w == 16) return region_w<16>(R, K, coef, in, bytes, out);
  if (w == -32) {  // unpacked w = 32
    switch (R) {
      case 1: region32u<1>(K, coef, in, bytes, out); return 0;
      case 4: region32u<4>(K, coef, in, bytes, out); return 0;
    }
  }
  return -1;
}

// rows -> planes -> rows must be the identity
extern "C" int gfs_transpose_roundtrip(int w, const uint32_t* rows, uint32_t* planes, uint32_t* back) {
  if (w == 32) {
    uint32_t r[32];
    std::memcpy(r, rows, sizeof r);
    leoec::gfs::transpose<32>(r);
    std::memcpy(planes, r, sizeof r);
    leoec::gfs::transpose<32>(r);
    std::memcpy(back, r, sizeof r);
    return 0;
  }
  uint32_t r[16];
  std::memcpy(r, rows, sizeof r);
  leoec::gfs::transpose<16>(r);
  std::memcpy(planes, r, sizeof r);
  leoec::gfs::transpose<16>(r);
  std::memcpy(back, r, sizeof r);
  return 0;
}
