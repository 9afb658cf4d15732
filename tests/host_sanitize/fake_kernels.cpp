// CPU implementations of the engine's launch() entry points (kernels.hpp),
// TEST INFRASTRUCTURE ONLY, for the host sanitizer harness: each launch is
// queued on the fake stream (hip/hip_runtime.h here) and computes exactly
// what the gfx950 kernel computes — the same shard geometry (object o's block
// at base + o * stride; bytes at or past `valid` read as zero and never
// written), so AddressSanitizer flags any shard the host side describes
// wrongly.  Not a product path: the engine's builds link kernels.hip.
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/leoec.h"
#include "../../leo_erasure_amd/csrc/codes.hpp"
#include "../../leo_erasure_amd/csrc/kernels.hpp"
#include "../../leo_erasure_amd/csrc/knobs.hpp"

namespace leoec {
namespace {

inline uint8_t rd(const Shard& s, uint64_t o, uint64_t pos) {
  return pos < s.valid ? s.base[o * s.stride + pos] : 0;
}
inline void wr(const Shard& s, uint64_t o, uint64_t pos, uint8_t v) {
  if (pos < s.valid) const_cast<uint8_t*>(s.base)[o * s.stride + pos] = v;
}

int enqueue(hipStream_t s, std::function<void()> f) {
  fake_stream(s)->push(std::move(f));
  return LEOEC_OK;
}

// bit i of c * 2^x in GF(2^w): the (i, x) entry of "multiply by c"
std::vector<uint8_t> mul_bits(const Field& F, uint32_t c, int w) {
  std::vector<uint8_t> m((size_t)w * w);
  uint32_t v = c;
  for (int x = 0; x < w; ++x) {
    for (int i = 0; i < w; ++i) m[(size_t)i * w + x] = (v >> i) & 1u;
    v = F.mul(v, 2);
  }
  return m;
}

// out packet `op` of output shard `so` ^= in packet `ip` of input shard `si`
void xor_packet(std::vector<uint8_t>& acc, const Shard& si, uint64_t o, uint64_t ip, uint64_t ps) {
  for (uint64_t b = 0; b < ps; ++b) acc[b] ^= rd(si, o, ip * ps + b);
}

}  // namespace

int launch(const GfApply& a, hipStream_t s) {
  return enqueue(s, [a] {
    const Field& F = field(a.w);
    const int wb = a.w / 8;
    std::vector<uint32_t> tab;  // w = 8: full product table per coefficient
    if (a.w == 8) {
      tab.resize((size_t)a.R * a.K * 256);
      for (int r = 0; r < a.R; ++r)
        for (int j = 0; j < a.K; ++j)
          for (int x = 0; x < 256; ++x)
            tab[((size_t)r * a.K + j) * 256 + x] = F.mul(a.coef[(size_t)r * a.K + j], (uint32_t)x);
    }
    for (uint64_t o = 0; o < a.nobj; ++o)
      for (int r = 0; r < a.R; ++r)
        for (uint64_t pos = 0; pos < a.block_size; pos += (uint64_t)wb) {
          uint32_t acc = 0;
          for (int j = 0; j < a.K; ++j) {
            uint32_t x = 0;
            for (int b = 0; b < wb; ++b) x |= (uint32_t)rd(a.in[j], o, pos + b) << (8 * b);
            const uint32_t c = a.coef[(size_t)r * a.K + j];
            acc ^= a.w == 8 ? tab[((size_t)r * a.K + j) * 256 + x] : F.mul(c, x);
          }
          for (int b = 0; b < wb; ++b) wr(a.out[r], o, pos + b, (uint8_t)(acc >> (8 * b)));
        }
  });
}

int launch(const GfBitApply& a, hipStream_t s) {
  return enqueue(s, [a] {
    const Field& F = field(a.w);
    const uint64_t ps = a.block_size / (uint64_t)a.w;
    std::vector<std::vector<uint8_t>> M((size_t)a.R * a.K);
    for (int r = 0; r < a.R; ++r)
      for (int j = 0; j < a.K; ++j) M[(size_t)r * a.K + j] = mul_bits(F, a.coef[(size_t)r * a.K + j], a.w);
    std::vector<uint8_t> acc(ps);
    for (uint64_t o = 0; o < a.nobj; ++o)
      for (int r = 0; r < a.R; ++r)
        for (int i = 0; i < a.w; ++i) {
          std::fill(acc.begin(), acc.end(), 0);
          for (int j = 0; j < a.K; ++j)
            for (int x = 0; x < a.w; ++x)
              if (M[(size_t)r * a.K + j][(size_t)i * a.w + x]) xor_packet(acc, a.in[j], o, x, ps);
          for (uint64_t b = 0; b < ps; ++b) wr(a.out[r], o, i * ps + b, acc[b]);
        }
  });
}

int launch(const BitApply& a, hipStream_t s) {
  return enqueue(s, [a] {
    const int w = a.w, cols = a.KB * w;
    const uint64_t ps = a.block_size / (uint64_t)w;
    std::vector<uint8_t> acc(ps);
    for (uint64_t o = 0; o < a.nobj; ++o)
      for (int op = 0; op < a.RB * w; ++op) {
        std::fill(acc.begin(), acc.end(), 0);
        for (int p = 0; p < cols; ++p)
          if (a.bits[(size_t)op * cols + p]) xor_packet(acc, a.in[p / w], o, p % w, ps);
        for (uint64_t b = 0; b < ps; ++b) wr(a.out[op / w], o, (op % w) * ps + b, acc[b]);
      }
  });
}

int launch(const LibDecApply& a, hipStream_t s) {
  return enqueue(s, [a] {
    const int w = a.w, k = a.k;
    BitMatrix B;
    if (liberation_coding_bitmatrix(k, w, &B)) return;
    const uint64_t ps = a.block_size / (uint64_t)w;
    // syndromes S_c = [c survives] C ^ B_{c,S} D_S for both coding blocks
    // (an absent shard reads as zero, as in the GPU kernel)
    std::vector<std::vector<uint8_t>> syn((size_t)2 * w, std::vector<uint8_t>(ps));
    std::vector<uint8_t> acc(ps);
    for (uint64_t o = 0; o < a.nobj; ++o) {
      for (int c = 0; c < 2; ++c) {
        for (int r = 0; r < w; ++r) {
          std::vector<uint8_t>& sy = syn[(size_t)c * w + r];
          std::fill(sy.begin(), sy.end(), 0);
          if (a.cod[c].base) xor_packet(sy, a.cod[c], o, r, ps);
          for (int j = 0; j < k; ++j)
            if (a.data[j].base)
              for (int x = 0; x < w; ++x)
                if (B.get(c * w + r, j * w + x)) xor_packet(sy, a.data[j], o, x, ps);
        }
      }
      for (size_t b = 0; b < a.out.size(); ++b)
        for (int x = 0; x < w; ++x) {
          std::fill(acc.begin(), acc.end(), 0);
          for (int sidx = 0; sidx < 2 * w; ++sidx)
            if ((a.mbits[b * 2 * w + sidx] >> (31 - x)) & 1u)
              for (uint64_t q = 0; q < ps; ++q) acc[q] ^= syn[sidx][q];
          for (uint64_t q = 0; q < ps; ++q) wr(a.out[b], o, x * ps + q, acc[q]);
        }
    }
  });
}

bool gfbit_supported(int w) { return w >= 2 && w <= 16; }
bool lib_dec_supported(int w) {
  return (w == 3 || w == 5 || w == 7 || w == 11 || w == 13) && knobs().lib_form != 0;
}

}  // namespace leoec
