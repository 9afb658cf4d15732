// gfs_core.hpp — bitsliced GF(2^w) multiply-accumulate for w = 16 and 32
// (vandrs / isars-style word codes: jerasure_matrix_encode and the decode
// maps over w = 16 / 32 words, c_src/rscoding.cpp:71,147,198).
//
// Why bitsliced.  Multiplication by a coefficient c is GF(2)-linear on the w
// bits of a word.  The byte-plane kernel (gfp_apply) applies it as 16 (w=32)
// or 4 (w=16) byte maps of 3 v_perm_b32 table lookups each, and v_perm runs
// at a quarter of the VALU rate on gfx950 (tools/valu_rate.hip: ~4.2 cycles
// per wave64 instruction, against ~2.3-2.6 for shifts, xor, v_bitop3).
// Here a lane transposes 32 words into w bit-planes (plane k = bit k of the
// 32 words), so that
//     c * x = XOR over the set bits t of c of  x * alpha^t
// becomes plain XORs of whole planes: x * alpha is a renaming of the planes
// plus 3 XORs (the polynomial's taps), and a set bit t of c costs w XORs
// into the accumulator: per coefficient and 32 words w/2 * w XORs on
// average, all full-rate, against 12 (w=32) or 6 (w=16) quarter-rate perms
// per word for the byte planes.  Bits are taken in pairs (t, t+1), one
// doubling step computing both x*alpha^t and x*alpha^(t+1); a pair with both
// bits set is one v_bitop3 (xor3) per register, so any nonzero pair costs
// one XOR per plane register (PairMasks).
//
// Layout of a lane's words ("rows").  w = 32: rows r[0..31] are the 32
// words.  w = 16: rows r[0..15] each hold two 16-bit words (low and high
// half).  transpose<W>() turns rows into planes and back (it is its own
// inverse).  Which word sits in which bit of a plane does not matter: the
// inverse transpose puts every word back where it came from.
//
// Portable C++ (host and device): tests/gfs_core_test.cpp checks it on the
// CPU against the oracle's field arithmetic.
#pragma once

#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define LEOEC_GFS_HD __host__ __device__ __forceinline__
#else
#define LEOEC_GFS_HD inline
#endif

namespace leoec {
namespace gfs {


// Field polynomial taps other than x^0 (gf-complete defaults, as
// codes.cpp's Field): w = 32: x^32 = x^22 + x^2 + x + 1 (0x400007);
// w = 16: x^16 = x^12 + x^3 + x + 1 (0x1100B).
LEOEC_GFS_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

template <int W>
constexpr int tap(int i) {
  return W == 32 ? (i == 0 ? 1 : i == 1 ? 2 : 22) : (i == 0 ? 1 : i == 1 ? 3 : 12);
}
constexpr int kTaps = 3;

// One stage of the recursive 32x32 bit transpose: rows k and k+j swap the
// bits of columns c+j and c (bit j of c clear).
template <int N, int J>
LEOEC_GFS_HD void swap_stage(uint32_t (&r)[N]) {
  constexpr uint32_t m = J == 16 ? 0x0000FFFFu
                         : J == 8 ? 0x00FF00FFu
                         : J == 4 ? 0x0F0F0F0Fu
                         : J == 2 ? 0x33333333u
                                  : 0x55555555u;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (k & J) continue;
    const uint32_t a = r[k], b = r[k + J];
    r[k] = (a & m) | ((b << J) & ~m);
    r[k + J] = (b & ~m) | ((a >> J) & m);
  }
}

// Rows <-> planes (self-inverse).  W = 16 rows are the packed form that the
// j = 16 stage of a 32-row transpose would produce from 32 zero-extended
// 16-bit words, so only the four lower stages run.
template <int W>
LEOEC_GFS_HD void transpose(uint32_t (&r)[W]) {
  if constexpr (W == 32) swap_stage<W, 16>(r);
  swap_stage<W, 8>(r);
  swap_stage<W, 4>(r);
  swap_stage<W, 2>(r);
  swap_stage<W, 1>(r);
}

// The bit pairs (T, T+1), T even, of a coefficient split three ways, bit T
// of each mask: both bits set (one v_bitop3 xor3 per register), only bit T,
// only bit T+1.  Three independent tests, so that every branch updates the
// accumulators in place (a three-way branch on one value made the compiler
// give each arm its own destination registers and copy them at the merge).
struct PairMasks {
  uint32_t both, lo, hi;
};
LEOEC_GFS_HD PairMasks pair_masks(uint32_t c) {
  constexpr uint32_t kEven = 0x55555555u;
  return PairMasks{c & (c >> 1) & kEven, c & ~(c >> 1) & kEven, (c >> 1) & ~c & kEven};
}

// One pair of coefficient bits (T, T+1), then the advance to P_{T+2} and
// the next pair: template recursion, so that every plane index is a
// compile-time constant (a runtime index would demote the arrays to scratch
// memory).  Logical plane k of x * alpha^T lives in pl[(k - T) mod W] (the
// doubling renames planes; only the tap planes are rewritten).
template <int W, int R, int T>
LEOEC_GFS_HD void mac_pair(uint32_t (&pl)[W], uint32_t (&acc)[R][W], const PairMasks (&c)[R],
                           uint32_t any) {
  constexpr int M = W - 1;
  // P_{T+1} = P_T * alpha: plane 0 = P_T[W-1], tap planes p = P_T[p-1] ^ P_T[W-1],
  // other planes k = P_T[k-1]
  const uint32_t top = pl[(M - T) & M];
  uint32_t tp[kTaps];
#pragma unroll
  for (int i = 0; i < kTaps; ++i) tp[i] = pl[(tap<W>(i) - 1 - T) & M] ^ top;
  // q0[k] = P_T[k], q1[k] = P_{T+1}[k]: register names only (no code), so
  // that no helper or lambda takes the plane array by reference (one left
  // un-inlined would put the arrays in scratch memory)
  uint32_t q0[W], q1[W];
#pragma unroll
  for (int k = 0; k < W; ++k) {
    q0[k] = pl[(k - T) & M];
    q1[k] = k == 0 ? top : pl[(k - 1 - T) & M];
  }
#pragma unroll
  for (int i = 0; i < kTaps; ++i) q1[tap<W>(i)] = tp[i];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    // wave-uniform: scalar branches
    if ((c[r].both >> T) & 1u) {
#pragma unroll
      for (int k = 0; k < W; ++k) acc[r][k] = xor3(acc[r][k], q0[k], q1[k]);
    }
    if ((c[r].lo >> T) & 1u) {
#pragma unroll
      for (int k = 0; k < W; ++k) acc[r][k] ^= q0[k];
    }
    if ((c[r].hi >> T) & 1u) {
#pragma unroll
      for (int k = 0; k < W; ++k) acc[r][k] ^= q1[k];
    }
  }
  if constexpr (T + 2 < W) {
    if ((any >> (T + 2)) == 0u) return;  // no coefficient has a higher bit
    // commit P_{T+1}'s tap planes (their registers held P_T[p-1]), advance
    // to P_{T+2}, next pair
#pragma unroll
    for (int i = 0; i < kTaps; ++i) pl[(tap<W>(i) - 1 - T) & M] = tp[i];
    const uint32_t top1 = pl[(M - T - 1) & M];  // P_{T+1}[W-1] = P_{T+2}[0]
#pragma unroll
    for (int i = 0; i < kTaps; ++i) pl[(tap<W>(i) - 2 - T) & M] ^= top1;
    mac_pair<W, R, T + 2>(pl, acc, c, any);
  }
}

// acc[r] ^= c[r] * x for R rows, x given as planes pl[] (destroyed).
template <int W, int R>
LEOEC_GFS_HD void mac(uint32_t (&pl)[W], uint32_t (&acc)[R][W], const uint32_t (&c)[R]) {
  PairMasks m[R];
  uint32_t any = 0u;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    m[r] = pair_masks(c[r]);
    any |= c[r];
  }
  mac_pair<W, R, 0>(pl, acc, m, any);
}

// ---------------------------------------------------------------------------
// w = 32 with 16 words per lane ("packed"): the W = 16 transpose applied to
// 16 words leaves register i holding plane i of the 16 words in its low half
// and plane i + 16 in its high half, so a lane needs 16 registers per value
// instead of 32 (4 output rows: 64 accumulator registers, 4 waves per SIMD
// instead of 2).  x * alpha in this layout: register i <- register i - 1 for
// i >= 1 (a renaming), register 0 <- register 15 with its halves swapped
// (new plane 0 = old plane 31, new plane 16 = old plane 15), then the taps:
// planes 1 and 2 (low halves of registers 1, 2) and plane 22 (high half of
// register 6) ^= new plane 0.  The accumulators keep the canonical layout,
// so accumulating is register-wise XOR as for W = 16.
LEOEC_GFS_HD uint32_t swap_halves(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(v, v, 16);
#else
  return (v >> 16) | (v << 16);
#endif
}

// The registers P_{T+1} differs in from P_T (logical indices 0, 1, 2, 6),
// given P_T's logical registers p[i] = pl[(i - T) mod 16].
struct P32Step {
  uint32_t r0, r1, r2, r6;
};
template <int T>
LEOEC_GFS_HD P32Step p32_step(const uint32_t (&pl)[16]) {
  P32Step n;
  const uint32_t top = pl[(15 - T) & 15];
  n.r0 = swap_halves(top);
  // tap terms: new plane 0 (= old plane 31, the high half of `top`) into the
  // low halves of registers 1 and 2, and into the high half of register 6
  // (plane 22): one v_bitop3 each, masks in scalar registers
  n.r1 = pl[(0 - T) & 15] ^ (n.r0 & 0x0000FFFFu);
  n.r2 = pl[(1 - T) & 15] ^ (n.r0 & 0x0000FFFFu);
  n.r6 = pl[(5 - T) & 15] ^ (top & 0xFFFF0000u);
  return n;
}

// ALLB (measurement only, not a code): every pair of every coefficient taken
// as "both bits set", with no tests — the same VALU work as the coefficient
// 0xFFFFFFFF without the scalar tests and branches.
template <int R, int T, bool ALLB = false>
LEOEC_GFS_HD void mac_p32_pair(uint32_t (&pl)[16], uint32_t (&acc)[R][16], const PairMasks (&c)[R],
                               uint32_t any) {
  const P32Step n = p32_step<T>(pl);
  uint32_t q0[16], q1[16];  // P_T, P_{T+1} (register names)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    q0[i] = pl[(i - T) & 15];
    q1[i] = pl[(i - 1 - T) & 15];
  }
  q1[0] = n.r0;
  q1[1] = n.r1;
  q1[2] = n.r2;
  q1[6] = n.r6;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if constexpr (ALLB) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[r][i] = xor3(acc[r][i], q0[i], q1[i]);
      continue;
    }
    // wave-uniform: scalar branches
    if ((c[r].both >> T) & 1u) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[r][i] = xor3(acc[r][i], q0[i], q1[i]);
    }
    if ((c[r].lo >> T) & 1u) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[r][i] ^= q0[i];
    }
    if ((c[r].hi >> T) & 1u) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[r][i] ^= q1[i];
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  // ALLB: keep the scheduler from hoisting work across pairs (without the
  // shipped form's branches it raised the kernel to 128 VGPRs and spilled)
  if constexpr (ALLB) __builtin_amdgcn_sched_barrier(0);
#endif
  if constexpr (T + 2 < 32) {
    if (!ALLB && (any >> (T + 2)) == 0u) return;  // no coefficient has a higher bit
    // commit P_{T+1} (logical register i of P_{T+1} lives in pl[(i - T - 1) mod 16])
    pl[(15 - T) & 15] = n.r0;
    pl[(0 - T) & 15] = n.r1;
    pl[(1 - T) & 15] = n.r2;
    pl[(5 - T) & 15] = n.r6;
    const P32Step n2 = p32_step<T + 1>(pl);  // P_{T+2}
    pl[(14 - T) & 15] = n2.r0;
    pl[(15 - T) & 15] = n2.r1;
    pl[(0 - T) & 15] = n2.r2;
    pl[(4 - T) & 15] = n2.r6;
    mac_p32_pair<R, T + 2, ALLB>(pl, acc, c, any);
  }
}

// acc[r] ^= c[r] * x over GF(2^32), 16 words per lane in the packed layout
// (transpose<16> of the 16 words; pl destroyed).
template <int R, bool ALLB = false>
LEOEC_GFS_HD void mac_p32(uint32_t (&pl)[16], uint32_t (&acc)[R][16], const uint32_t (&c)[R]) {
  PairMasks m[R];
  uint32_t any = 0u;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    m[r] = pair_masks(c[r]);
    any |= c[r];
  }
  mac_p32_pair<R, 0, ALLB>(pl, acc, m, any);
}

}  // namespace gfs
}  // namespace leoec
