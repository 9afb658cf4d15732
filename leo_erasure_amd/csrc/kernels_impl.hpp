// kernels_impl.hpp — gfx950 (CDNA4) kernels of the erasure-coding engine and
// their launch templates.  Included by kernels.hip (dispatch, w=16/32 and
// bitmatrix instances) and gf8_inst.hip (GF(2^8) instances, one translation
// unit per input count K so the 128 unrolled variants build in parallel).
//
// The work is memory-bound byte / XOR arithmetic: no MFMA and no LDS.  Each
// lane owns one 16-byte column of a block and walks down the K input blocks
// with global_load_dwordx4 (one wave reads 1 KiB contiguous per block: fully
// coalesced), keeps its R output columns in VGPRs and stores each once, so
// every input byte is read from HBM once and every output byte written once.
//
// GF(2^8) multiply by a wave-uniform constant c uses v_perm_b32 as an 8-entry
// byte-table lookup (four lookups per instruction):
//     c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
// with T0[i] = c*i, T1[i] = c*(i<<3), T2[i] = c*(i<<6) (poly 0x11D).  The three
// selector dwords of a data dword are shared by every output row; per
// coefficient a dword costs 3 v_perm + v_bitop3 (xor3) + v_xor.  Coefficients
// 0 and 1 take a scalar branch (skip / plain xor).  The 5 table dwords per
// coefficient are kernel arguments, read by s_load into SGPRs.
//
// GF(2^16) / GF(2^32) use shift-and-add: x*2^b is formed once per input word
// and masked into every row whose coefficient has bit b (v_bitop3 a^(b&c)).
//
// Bitmatrix codes (cauchyrs, liberation) are a GF(2) matrix over packets of
// block_size / w bytes: out packet o ^= in packet p & mask(o, p), the 0/~0
// masks taken from one uniform bit word per input packet.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/leoec.h"
#include "kernels.hpp"
#include "tile_maps.hpp"

namespace leoec {
namespace detail {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr uint32_t kTileBytes = kThreads * 16;  // one 16-byte column per lane
constexpr int kMaxK = 16;                       // input blocks per launch
constexpr int kMaxR = 4;                        // GF output blocks per launch
constexpr int kMaxPk = 32;                      // bitmatrix output packets per launch

struct DevShard {
  const uint8_t* base;
  uint64_t stride;
  uint32_t valid;
  uint32_t pad;
};

// One launch covers objects [o0, o0+no) and output rows / input columns
// [r0, r0+nr) x [j0, j0+nk) of the plan; tiles = 4 KiB tiles per block.
struct Chunk {
  int r0, nr, j0, nk;
  uint64_t o0, no;
  uint32_t tiles;
};

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// 16-byte global access; NT = non-temporal (data streamed once: measured
// +9 % on the RS(10,4) encode, tools/kvariants.py).
template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<const u32x4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = v;
}

// Raw buffer resource over [p, p + 4 GiB): loads/stores then take one shared
// 32-bit VGPR offset plus a per-block SGPR base instead of a 64-bit VGPR
// address per access (gfx9 dword3 = 0x00020000).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0xFFFFFFFF, 0x00020000);
}

// Bytes of v at index >= n (0 <= n < 16) cleared.
__device__ __forceinline__ u32x4 keep_first(u32x4 v, uint32_t n) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t lo = 4u * e;
    const uint32_t m = n >= lo + 4u ? 0xFFFFFFFFu : (n <= lo ? 0u : (1u << (8u * (n - lo))) - 1u);
    v[e] &= m;
  }
  return v;
}

// One input block of a launch with its column of coefficients: 64 bytes, so
// that a kernel's input loop fetches everything it needs for an input with
// one scalar load, one input ahead (the scalar loads are then waited for
// behind a whole input's arithmetic instead of in front of it).  Used by
// gfs_apply and gfb2_apply.
struct InCol {
  const uint8_t* base;
  uint64_t stride;
  uint32_t valid;
  uint32_t pad;
  uint32_t coef[kMaxR];  // coef[r] = c_rj
  uint32_t pad2[6];
};
static_assert(sizeof(InCol) == 64, "InCol is one 64-byte scalar load");

// Raw buffer resource over one shard of object o whose range ends at `valid`
// rounded up to a whole chunk of `chunk` bytes (a power of two): loads of
// chunks past it read as zeros without a memory access, so a kernel's loads
// can be unconditional (a per-lane branch around a load makes the compiler
// wait for every outstanding load, prefetches included, at the merge), and
// the chunk straddling `valid` is cleared by the kernel.  valid 0 = empty.
// valid <= 2^32 - 16 (launchers refuse blocks of 4 GiB); no clamp, which the
// compiler would turn into a vector saturating add, making the resource
// divergent (a waterfall loop around every load).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t shard_rsrc(const uint8_t* base, uint64_t stride,
                                                             uint32_t valid, uint64_t o,
                                                             uint32_t chunk) {
  // the arguments are wave-uniform; readfirstlane says so to the compiler
  // where a loop-carried copy of one ended up in a VGPR (free for SGPRs)
  const uint32_t nrec = __builtin_amdgcn_readfirstlane((valid + chunk - 1u) & ~(chunk - 1u));
  const uint64_t addr = (uint64_t)(uintptr_t)(base + o * stride);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)addr);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((uintptr_t)(((uint64_t)hi << 32) | lo)), 0, nrec, 0x00020000);
}

// Guarded load for tiles that cross a block's valid length: a chunk whose
// first byte is valid is read whole (an aligned 16-byte chunk never crosses a
// page) and its bytes past `valid` cleared; chunks past `valid` are not read.
__device__ __forceinline__ u32x4 load_guarded(const uint8_t* p, uint32_t off, uint32_t valid) {
  u32x4 v = {0u, 0u, 0u, 0u};
  if (off < valid) v = ld16<true>(p + off);
  if (off + 16u > valid) v = keep_first(v, off < valid ? valid - off : 0u);
  return v;
}

// Guarded store: never writes a byte at or past `valid`.
__device__ __forceinline__ void store_guarded(uint8_t* p, uint32_t off, uint32_t valid, u32x4 v) {
  if (off + 16u <= valid) {
    st16<true>(p + off, v);
  } else if (off < valid) {
    const uint32_t n = valid - off;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((uint32_t)i < n) p[off + i] = (uint8_t)(v[i >> 2] >> (8 * (i & 3)));
  }
}

// ===========================================================================
// GF(2^8): K inputs x R outputs, fully unrolled.
template <int K, int R>
struct Gf8Args {
  DevShard in[K];
  DevShard out[R];
  uint32_t tab[R][K][5];  // T0 lo, T0 hi, T1 lo, T1 hi, T2
  uint64_t one;           // bit r*K+j set: coefficient is 1
  uint64_t zero;          // bit r*K+j set: coefficient is 0
  uint32_t tiles;         // tiles per object
  uint32_t vmin;          // min valid over all shards of the launch
  uint32_t total_tiles;   // tiles of the launch (persistent form)
  uint32_t nobj;          // objects of the launch
  uint32_t tmap;          // workgroup -> tile order: 0 tile-major, 1 object-major,
                          // 2 tiles of an object visited with stride tperm (coprime),
                          // 3 xcd_obj_map (shipped for <= kObjMapMaxTiles tiles),
                          // 4 xcd_obj_map over groups of tperm consecutive tiles of
                          //   the object-major tile order (stripe segments per XCD)
  uint32_t tperm;
};

// Kernel shape / policy knobs (the engine ships kGf8Default; the others exist
// for A/B measurement through LEOEC_GF8_VARIANT, see tools/kvariants.py).
struct Gf8Opt {
  int xmap;     // compiled-in workgroup -> (object, tile) map: 0 none (the
                // launcher then picks tmap 3 = xcd_obj_map at run time), 1 xcd_group,
                // 2 xcd_obj_map always
  int cpt;      // 16-byte columns per lane (tile = 4 KiB * cpt per block)
  bool nt;      // non-temporal loads / stores (streamed once, never re-read)
  int branchy;  // 1: scalar branch on coefficients 0 / 1; 0: all tables, xor3-paired;
                // -1: pick per launch from the coefficients
  bool copy;    // measurement only: same traffic, XOR instead of GF multiply
  bool lds;     // perm tables staged in LDS (VGPR operands) instead of SGPRs
  int waves;    // minimum waves per SIMD requested from the register allocator
};
constexpr Gf8Opt kGf8Default{0, 1, true, 0, false, true, 5};


// One tile of the GF(2^8) map for columns already loaded in d.
//  BRANCHY: coefficient 1 -> plain xor, 0 -> skip (scalar branches), others
//           3 perm + xor3 + xor;
//  !BRANCHY: every coefficient through its tables, with the 3K perm outputs
//           of a row folded pairwise by xor3 (1.5 ops per coefficient).
// Per-coefficient v_perm tables staged in LDS: [t0 lo, t0 hi, t1 lo, t1 hi]
// and [t2, -, -, -] (32 bytes per coefficient, 16-byte aligned).
template <int K, int R>
struct Gf8Lds {
  u32x4 t[R * K][2];
};

template <int K, int R, int CPT, bool BRANCHY, bool COPY, bool LDS>
__device__ __forceinline__ void gf8_tile(const Gf8Args<K, R>& a, const Gf8Lds<K, R>& lds,
                                         const u32x4 (&d)[CPT][K], u32x4 (&acc)[CPT][R]) {
  u32x4 pend[CPT][R];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (COPY) {
#pragma unroll
      for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[c][r] ^= d[c][j];
      continue;
    }
    uint32_t s0[CPT][4], s1[CPT][4], s2[CPT][4];
#pragma unroll
    for (int c = 0; c < CPT; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t x = d[c][j][e];
        s0[c][e] = x & 0x07070707u;
        s1[c][e] = (x >> 3) & 0x07070707u;
        s2[c][e] = (x >> 6) & 0x03030303u;
      }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int bit = r * K + j;
      if (BRANCHY && ((a.one >> bit) & 1)) {
#pragma unroll
        for (int c = 0; c < CPT; ++c) acc[c][r] ^= d[c][j];
      } else if (!BRANCHY || !((a.zero >> bit) & 1)) {
        uint32_t t0l, t0h, t1l, t1h, t2;
        if (LDS) {  // VGPR operands: no SGPR pressure, no constant-bus moves
          const u32x4 t = lds.t[r * K + j][0];
          t0l = t[0]; t0h = t[1]; t1l = t[2]; t1h = t[3];
          t2 = lds.t[r * K + j][1][0];
        } else {
          t0l = a.tab[r][j][0]; t0h = a.tab[r][j][1];
          t1l = a.tab[r][j][2]; t1h = a.tab[r][j][3];
          t2 = a.tab[r][j][4];
        }
#pragma unroll
        for (int c = 0; c < CPT; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t p0 = perm(t0h, t0l, s0[c][e]);
            const uint32_t p1 = perm(t1h, t1l, s1[c][e]);
            const uint32_t p2 = perm(t2, t2, s2[c][e]);
            if (BRANCHY) {
              acc[c][r][e] = xor3(acc[c][r][e], p0, p1) ^ p2;
            } else if ((j & 1) == 0) {  // static after unrolling
              acc[c][r][e] = xor3(acc[c][r][e], p0, p1);
              pend[c][r][e] = p2;
            } else {
              acc[c][r][e] = xor3(acc[c][r][e], pend[c][r][e], p0);
              acc[c][r][e] = xor3(acc[c][r][e], p1, p2);
            }
          }
      }
    }
  }
  if (!BRANCHY && !COPY && (K & 1)) {
#pragma unroll
    for (int c = 0; c < CPT; ++c)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[c][r] ^= pend[c][r];
  }
}

// As gf8_tile (paired form) for a matrix whose row 0 and column 0 are all
// ones (every vandrs encode matrix): those K+R-1
// coefficients contribute the data word itself (one term) instead of three
// table lookups; every term of a row is folded pairwise into xor3 with the
// pairing worked out at compile time.  The launcher checks the property.
template <int K, int R, int CPT, bool LDS>
__device__ __forceinline__ void gf8_tile_ones(const Gf8Lds<K, R>& lds, const u32x4 (&d)[CPT][K],
                                              u32x4 (&acc)[CPT][R]) {
  u32x4 pend[CPT][R];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    uint32_t s0[CPT][4], s1[CPT][4], s2[CPT][4];
    if (j > 0) {
#pragma unroll
      for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t x = d[c][j][e];
          s0[c][e] = x & 0x07070707u;
          s1[c][e] = (x >> 3) & 0x07070707u;
          s2[c][e] = (x >> 6) & 0x03030303u;
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool one = r == 0 || j == 0;
      int pos = 0;  // terms of row r before coefficient j (folds to a constant)
#pragma unroll
      for (int jj = 0; jj < j; ++jj) pos += (r == 0 || jj == 0) ? 1 : 3;
      uint32_t t0l = 0, t0h = 0, t1l = 0, t1h = 0, t2 = 0;
      if (!one) {
        const u32x4 t = lds.t[r * K + j][0];
        t0l = t[0]; t0h = t[1]; t1l = t[2]; t1h = t[3];
        t2 = lds.t[r * K + j][1][0];
      }
#pragma unroll
      for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uint32_t term[3];
          int n = 1;
          if (one) {
            term[0] = d[c][j][e];
          } else {
            term[0] = perm(t0h, t0l, s0[c][e]);
            term[1] = perm(t1h, t1l, s1[c][e]);
            term[2] = perm(t2, t2, s2[c][e]);
            n = 3;
          }
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            if (i >= n) break;
            if (((pos + i) & 1) == 0) pend[c][r][e] = term[i];
            else acc[c][r][e] = xor3(acc[c][r][e], pend[c][r][e], term[i]);
          }
        }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int tot = 0;
#pragma unroll
    for (int jj = 0; jj < K; ++jj) tot += (r == 0 || jj == 0) ? 1 : 3;
    if (tot & 1) {
#pragma unroll
      for (int c = 0; c < CPT; ++c) acc[c][r] ^= pend[c][r];
    }
  }
}

template <int K, int R, int CPT, bool NT, uint32_t CS = kTileBytes, bool BUF = false>
__device__ __forceinline__ void gf8_load(const Gf8Args<K, R>& a, uint64_t o, uint32_t off,
                                         bool full, u32x4 (&d)[CPT][K]) {
  constexpr uint32_t kTileBytes = CS;
  if (full && BUF) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const auto rs = buf_rsrc(a.in[j].base + o * a.in[j].stride);
#pragma unroll
      for (int c = 0; c < CPT; ++c)
        d[c][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + c * kTileBytes, 0, NT ? 2 : 0);
    }
  } else if (full) {
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int c = 0; c < CPT; ++c)
        d[c][j] = ld16<NT>(a.in[j].base + o * a.in[j].stride + off + c * kTileBytes);
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int c = 0; c < CPT; ++c)
        d[c][j] = load_guarded(a.in[j].base + o * a.in[j].stride, off + c * kTileBytes,
                               a.in[j].valid);
  }
}

template <int K, int R, bool ACC, int CPT, bool NT, uint32_t CS = kTileBytes>
__device__ __forceinline__ void gf8_init_store(const Gf8Args<K, R>& a, uint64_t o, uint32_t off,
                                               u32x4 (&acc)[CPT][R]) {
  constexpr uint32_t kTileBytes = CS;
#pragma unroll
  for (int c = 0; c < CPT; ++c)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      acc[c][r] = u32x4{0u, 0u, 0u, 0u};
      if (ACC)
        acc[c][r] = load_guarded(a.out[r].base + o * a.out[r].stride, off + c * kTileBytes,
                                 a.out[r].valid);
    }
}

template <int K, int R, int CPT, bool NT, uint32_t CS = kTileBytes, bool BUF = false>
__device__ __forceinline__ void gf8_store(const Gf8Args<K, R>& a, uint64_t o, uint32_t off,
                                          bool full, const u32x4 (&acc)[CPT][R]) {
  constexpr uint32_t kTileBytes = CS;
  if (full && BUF) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const auto rs = buf_rsrc(a.out[r].base + o * a.out[r].stride);
#pragma unroll
      for (int c = 0; c < CPT; ++c)
        __builtin_amdgcn_raw_buffer_store_b128(acc[c][r], rs, off + c * kTileBytes, 0, NT ? 2 : 0);
    }
  } else if (full) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int c = 0; c < CPT; ++c)
        st16<NT>(const_cast<uint8_t*>(a.out[r].base) + o * a.out[r].stride + off + c * kTileBytes,
                 acc[c][r]);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int c = 0; c < CPT; ++c)
        store_guarded(const_cast<uint8_t*>(a.out[r].base) + o * a.out[r].stride,
                      off + c * kTileBytes, a.out[r].valid, acc[c][r]);
  }
}

// One workgroup per tile (PIPE = false), or a persistent grid that walks the
// tiles and issues the loads of its next tile before computing the current
// one (PIPE = true).
// Workgroup-id remaps (xcd_group, xcd_obj_map): tile_maps.hpp, CPU-tested
// for bijectivity (tests/test_tile_maps.py).
//
// Object-interleaved XCD map: with the dispatcher dealing workgroup ids
// round-robin over the 8 XCDs, give XCD x the objects o = x (mod 8) with all
// of an object's `tiles` tiles in order, so neighbouring tiles (which share
// the partial cache lines of packets that start mid-line) meet in one L2 at
// about the same time, while the 8 XCDs still work on neighbouring objects.
// Ids past the last whole group of 8 objects keep their place.  Used when an
// object has at most kObjMapMaxTiles tiles (1 MiB objects: +2-3 % on gf8,
// +1-2 % on cauchyrs, +4-8 % on liberation); with many tiles per object
// (objects of 4 MiB and up) it measured 2-4 % slower than dispatch order.
constexpr uint32_t kObjMapMaxTiles = 64;
// Blocks of at least kSegMapMinTiles tiles (32 MiB objects: 3,277 tiles of
// 1 KiB; 64 MiB: 6,554) run gf8_apply under tile map 4 with groups of
// kSegMapGroup tiles: XCD x takes every 8th run of 128 consecutive tiles
// (128 KiB of each block), so each L2 streams whole 128 KiB stretches of the
// 14 blocks instead of every 8th KiB.  RS(10,4,8), one process each
// (profiles/r02_v13_ab_tmap4_*.log): 64 x 64 MiB 0.720 / 0.734 -> 0.743 /
// 0.744 of HBM peak (encode / decode), 128 x 32 MiB 0.722 / 0.736 -> 0.743 /
// 0.742; 16 MiB (1,639 tiles) unchanged and 4 MiB (410 tiles) 1 % slower, so
// smaller blocks keep id order.
constexpr uint32_t kSegMapMinTiles = 2048;
constexpr uint32_t kSegMapGroup = 128;

// One workgroup of WG threads per tile (PIPE = false), or a persistent grid
// that walks the tiles and issues the loads of its next tile before
// computing the current one (PIPE = true).
//  EARLY: the tile's loads are issued before the coefficient tables are
//         staged into LDS (the staging and its barrier then overlap the
//         loads' flight instead of delaying them; the barrier waits for LDS
//         only, never for the loads).
template <int K, int R, bool ACC, int CPT, bool NT, bool BRANCHY, bool COPY, bool PIPE, bool LDS,
          int WAVES, int WG, int XMAP, bool BUF = false, bool ONES = false, bool EARLY = false>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(WAVES, 8)))
gf8_apply(const Gf8Args<K, R> a) {
  constexpr uint32_t CS = (uint32_t)WG * 16u;  // bytes of one column group
  constexpr uint32_t TB = CS * CPT;
  // With one column per lane the launcher may use fewer lanes than WG (the
  // workgroup size is then the tile width: 64 lanes = 1 KiB tiles, chosen for
  // large blocks); CPT > 1 forms always launch WG lanes.
  const uint32_t TBr = CPT == 1 ? blockDim.x * 16u : TB;
  __shared__ Gf8Lds<K, R> lds;
  auto stage = [&]() {
    for (uint32_t i = threadIdx.x; i < (uint32_t)(R * K); i += blockDim.x) {
      const uint32_t* t = a.tab[i / K][i % K];
      lds.t[i][0] = u32x4{t[0], t[1], t[2], t[3]};
      lds.t[i][1] = u32x4{t[4], 0u, 0u, 0u};
    }
  };
  constexpr bool kEarly = EARLY && LDS && !PIPE;
  if (LDS && !kEarly) {
    stage();
    __syncthreads();
  }
  if (!PIPE) {
    const uint32_t b = XMAP == 1 ? xcd_group(blockIdx.x, gridDim.x)
                       : (XMAP == 2 || a.tmap == 3) ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles)
                       : a.tmap == 4                ? xcd_obj_map(blockIdx.x, gridDim.x, a.tperm)
                                                    : blockIdx.x;
    uint32_t obj, tile;
    if (a.tmap == 1) {
      tile = b / a.nobj;
      obj = b - tile * a.nobj;
    } else {
      obj = b / a.tiles;
      tile = b - obj * a.tiles;
      if (a.tmap == 2) tile = (uint32_t)(((uint64_t)tile * a.tperm) % a.tiles);
    }
    const uint32_t t0 = tile * TBr;
    const uint32_t off = t0 + threadIdx.x * 16u;
    const bool full = t0 + TBr <= a.vmin;  // wave-uniform
    u32x4 d[CPT][K];
    gf8_load<K, R, CPT, NT, CS, BUF>(a, obj, off, full, d);
    if (kEarly) {
      stage();
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: the LDS writes, not the loads
      __builtin_amdgcn_s_barrier();
    }
    u32x4 acc[CPT][R];
    gf8_init_store<K, R, ACC, CPT, NT, CS>(a, obj, off, acc);
    if (ONES && LDS && !COPY)
      gf8_tile_ones<K, R, CPT, LDS>(lds, d, acc);
    else
      gf8_tile<K, R, CPT, BRANCHY, COPY, LDS>(a, lds, d, acc);
    gf8_store<K, R, CPT, NT, CS, BUF>(a, obj, off, full, acc);
    return;
  }
  const uint32_t total = a.total_tiles;
  uint32_t g = blockIdx.x;
  if (g >= total) return;
  u32x4 nxt[CPT][K];
  uint32_t obj = g / a.tiles;
  uint32_t t0 = (g - obj * a.tiles) * TB;
  bool full = t0 + TB <= a.vmin;
  gf8_load<K, R, CPT, NT, CS>(a, obj, t0 + threadIdx.x * 16u, full, nxt);
  while (true) {
    u32x4 d[CPT][K];
#pragma unroll
    for (int c = 0; c < CPT; ++c)
#pragma unroll
      for (int j = 0; j < K; ++j) d[c][j] = nxt[c][j];
    const uint32_t cobj = obj, coff = t0 + threadIdx.x * 16u;
    const bool cfull = full;
    g += gridDim.x;
    const bool more = g < total;
    if (more) {
      obj = g / a.tiles;
      t0 = (g - obj * a.tiles) * TB;
      full = t0 + TB <= a.vmin;
      gf8_load<K, R, CPT, NT, CS>(a, obj, t0 + threadIdx.x * 16u, full, nxt);
    }
    u32x4 acc[CPT][R];
    gf8_init_store<K, R, ACC, CPT, NT, CS>(a, cobj, coff, acc);
    gf8_tile<K, R, CPT, BRANCHY, COPY, LDS>(a, lds, d, acc);
    gf8_store<K, R, CPT, NT, CS>(a, cobj, coff, cfull, acc);
    if (!more) break;
  }
}

// ===========================================================================
// Bitmatrix (GF(2)) over packets of ps bytes.
struct BitArgs {
  DevShard in[kMaxK];
  DevShard out[kMaxPk];        // one per output packet, base already at the packet
  uint32_t bits[kMaxK * 32];   // per input packet: bit (31 - o) set => feeds output packet o
  int w;
  int KP;                      // input packets = input blocks * w
  uint32_t ps;                 // packet bytes
  uint32_t tiles;              // tiles per object (over one packet)
};

// BR: per (input packet, output packet) pair a wave-uniform branch on the
// bitmatrix bit (scalar unit) and a plain xor when set, instead of a masked
// xor for every pair (vector unit).  PFD: loads of the next PFD input packets
// are kept in flight while one is applied (a ring of PFD+1 registers).  A
// streaming kernel needs ~50 KB in flight per CU to cover HBM latency; with
// one packet at a time a wave holds only 1 KiB.
template <int RO, bool ACC, bool BR = false, int PFD = 1, int XMAP = 0>
__global__ void __launch_bounds__(kThreads) bit_apply(const BitArgs a) {
  constexpr int RS = PFD + 1;
  const uint32_t bid = XMAP == 1 ? xcd_group(blockIdx.x, gridDim.x)
                       : XMAP == 2 ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t off = tile * kTileBytes + threadIdx.x * 16u;
  if (off >= a.ps) return;
  const uint64_t o64 = obj;
  u32x4 acc[RO];
#pragma unroll
  for (int o = 0; o < RO; ++o) {
    acc[o] = u32x4{0u, 0u, 0u, 0u};
    if (ACC) acc[o] = load_guarded(a.out[o].base + o64 * a.out[o].stride, off, a.out[o].valid);
  }
  auto load_packet = [&](int p) {
    const int blk = p / a.w, x = p - blk * a.w;  // wave-uniform
    const uint32_t pk = (uint32_t)x * a.ps;
    const uint32_t bv = a.in[blk].valid;
    return load_guarded(a.in[blk].base + o64 * a.in[blk].stride + pk, off, bv > pk ? bv - pk : 0u);
  };
  u32x4 ring[RS];
#pragma unroll
  for (int u = 0; u < PFD; ++u) ring[u] = u < a.KP ? load_packet(u) : u32x4{0u, 0u, 0u, 0u};
  for (int p0 = 0; p0 < a.KP; p0 += RS) {
#pragma unroll
    for (int u = 0; u < RS; ++u) {
      const int p = p0 + u;
      if (p < a.KP) {
        if (p + PFD < a.KP) ring[(u + PFD) % RS] = load_packet(p + PFD);
        const u32x4 v = ring[u];
        const uint32_t bits = a.bits[p];
#pragma unroll
        for (int o = 0; o < RO; ++o) {
          if (BR) {
            if ((bits << o) & 0x80000000u) {
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[o][e] ^= v[e];
            }
          } else {
            const uint32_t m = (uint32_t)((int32_t)(bits << o) >> 31);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[o][e] ^= v[e] & m;
          }
        }
      }
    }
  }
#pragma unroll
  for (int o = 0; o < RO; ++o) {
    uint8_t* p = const_cast<uint8_t*>(a.out[o].base);
    if (p != nullptr) store_guarded(p + o64 * a.out[o].stride, off, a.out[o].valid, acc[o]);
  }
}

// ===========================================================================
// Liberation encode (m = 2, k <= w, w prime): the bitmatrix of
// liberation_coding_bitmatrix (codes.cpp; SURVEY Appendix A.4,
// c_src/liberationcoding.cpp:39) has 2kw + k - 1 ones out of 2kw * w, so the
// masked kernel above spends ~93 % of its xors on zero bits.  Here the
// structure is compiled in: with the block index j unrolled (k <= W),
//   P[x]             ^= D(j, x)
//   Q[(x - j) mod W] ^= D(j, x)
//   Q[y]             ^= D(j, (y + j - 1) mod W),  y = j (W - 1) / 2 mod W, j > 0
// all with static register indices: 2 (or 3) xors per input packet dword,
// no branches.  The launcher checks the plan's bits against this structure
// and uses the generic kernel otherwise.  Packets are applied in (j, x) order
// with the loads of the next LA packets in flight (a ring of registers).
struct LibArgs {
  DevShard in[kMaxK];
  DevShard out[2];  // coding blocks P, Q (base at the block)
  int k;
  uint32_t ps;      // packet bytes
  uint32_t tiles;   // tiles per object (over one packet)
  uint32_t vmin;    // min valid over inputs and outputs
  uint32_t xmap;    // 1: xcd_obj_map
};

// Register budget: the 2W accumulators plus the ring; without a bound the
// scheduler hoists every load of the unrolled body (up to 256 VGPRs, one
// wave per SIMD).
constexpr int lib_waves(int w) { return w <= 7 ? 4 : w <= 11 ? 3 : 2; }

// TW: lanes per workgroup = 16-byte columns per tile.  lib_apply ships with
// 64 lanes (1 KiB of every packet per tile, kernels.hip kLibLanes); 256
// lanes (4 KiB tiles) and the other look-ahead depths are measurement-build
// forms.  (lib_dec_apply still ships with 256 lanes.)
template <int W, int LA, int TW = kThreads>
__global__ void __launch_bounds__(TW) __attribute__((amdgpu_waves_per_eu(lib_waves(W), 8)))
lib_apply(const LibArgs a) {
  constexpr int RS = LA + 1;  // ring of packet registers: LA loads in flight
  constexpr uint32_t kTileBytes = TW * 16u;
  const uint32_t bid = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t t0 = tile * kTileBytes;
  const uint32_t off = t0 + threadIdx.x * 16u;
  if (off >= a.ps) return;
  const uint64_t o64 = obj;
  // wave-uniform: the tile lies inside the packet and inside every shard's
  // valid bytes (the last packet of a block is the furthest)
  const bool full = t0 + kTileBytes <= a.ps &&
                    (uint64_t)(W - 1) * a.ps + t0 + kTileBytes <= (uint64_t)a.vmin;
  auto load = [&](int j, int x) {
    const uint8_t* b = a.in[j].base + o64 * a.in[j].stride;
    const uint32_t pk = (uint32_t)x * a.ps;
    if (full) return ld16<true>(b + pk + off);
    const uint32_t v = a.in[j].valid;
    return load_guarded(b + pk, off, v > pk ? v - pk : 0u);
  };
  u32x4 P[W], Q[W], ring[RS];
#pragma unroll
  for (int x = 0; x < W; ++x) P[x] = Q[x] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int q = 0; q < LA; ++q) {
    ring[q] = u32x4{0u, 0u, 0u, 0u};
    if (q < W * W && q / W < a.k) ring[q] = load(q / W, q % W);
  }
#pragma unroll
  for (int j = 0; j < W; ++j) {
    if (j >= a.k) break;
    const int y = (j * ((W - 1) / 2)) % W;  // Q row of block j's extra one
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const int p = j * W + x, q = p + LA;  // packet applied / packet loaded
      if (q < W * W && q / W < a.k) ring[q % RS] = load(q / W, q % W);
      const u32x4 v = ring[p % RS];
      P[x] ^= v;
      Q[(x - j + W) % W] ^= v;
      if (j > 0 && x == (y + j - 1) % W) Q[y] ^= v;
    }
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint8_t* b = const_cast<uint8_t*>(a.out[r].base) + o64 * a.out[r].stride;
    const uint32_t v = a.out[r].valid;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint32_t pk = (uint32_t)x * a.ps;
      const u32x4 acc = r == 0 ? P[x] : Q[x];
      if (full) st16<true>(b + pk + off, acc);
      else store_guarded(b + pk, off, v > pk ? v - pk : 0u, acc);
    }
  }
}

// ===========================================================================
// Liberation decode / data repair through syndromes.  The decoding
// bitmatrix G_S^-1 of the survivor set S is ~45 % ones (an inverse), so the
// masked kernel pays 2w v_bitop3 per input packet dword and is VALU-bound at
// w >= 11.  Instead, with E the erased data blocks and C the coding blocks
// in S (|C| = |E| <= 2):
//   syndrome  S_c = c ^ sum over surviving data j of B_cj D_j   (c in C)
//             (the liberation encode structure of lib_apply, static)
//   data      D_E = (B_CE)^-1 S_C                                (eW x eW)
// B_CE^-1 is built on the host; its rows for the wanted blocks come as one
// mask word per syndrome packet.  For every input the result is the one
// linear map G_S^-1 restricted to the wanted rows (the survivors determine
// the codeword uniquely), so outputs equal the generic path's bit for bit.
struct LibDecArgs {
  DevShard data[kMaxK];   // data block j (base nullptr if erased)
  DevShard cod[2];        // P, Q (base nullptr if not a survivor)
  DevShard out[2];        // wanted (erased data) blocks
  uint32_t mbits[2][32];  // [wanted block][syndrome packet s: P 0..W-1, Q W..2W-1]:
                          // bit (31 - x) set => feeds output packet x
  int k;
  int nout;
  uint32_t ps;
  uint32_t tiles;
  uint32_t vmin;          // min valid over every shard read or written
  uint32_t xmap;          // 1: xcd_obj_map
};

constexpr int lib_dec_waves(int w) { return w <= 5 ? 4 : w <= 11 ? 3 : 2; }

// TW: lanes per workgroup = 16-byte columns per tile (as lib_apply).
template <int W, int TW = kThreads>
__global__ void __launch_bounds__(TW) __attribute__((amdgpu_waves_per_eu(lib_dec_waves(W), 8)))
lib_dec_apply(const LibDecArgs a) {
  constexpr uint32_t kTileBytes = TW * 16u;
  const uint32_t bid = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t t0 = tile * kTileBytes;
  const uint32_t off = t0 + threadIdx.x * 16u;
  if (off >= a.ps) return;
  const uint64_t o64 = obj;
  const bool full = t0 + kTileBytes <= a.ps &&
                    (uint64_t)(W - 1) * a.ps + t0 + kTileBytes <= (uint64_t)a.vmin;
  auto load = [&](const DevShard& sh, int x) {
    const uint8_t* b = sh.base + o64 * sh.stride;
    const uint32_t pk = (uint32_t)x * a.ps;
    if (full) return ld16<true>(b + pk + off);
    const uint32_t v = sh.valid;
    return load_guarded(b + pk, off, v > pk ? v - pk : 0u);
  };
  // One static packet stream: P (W packets), Q (W), then data blocks 0..k-1,
  // with the loads of the next LA packets in flight (as lib_apply).  Absent
  // shards (P or Q not a survivor, erased data blocks) read as zero without
  // a memory access, so the stream's register indices stay static.
  constexpr int LA = 2, RS = LA + 1, NP = (W + 2) * W;
  auto shard_of = [&](int blk) -> const DevShard& {  // blk: 0 P, 1 Q, 2 + j data j
    return blk < 2 ? a.cod[blk] : a.data[blk - 2];
  };
  auto fetch = [&](int q) {
    const int blk = q / W;
    const DevShard& sh = shard_of(blk);
    if ((blk >= 2 && blk - 2 >= a.k) || sh.base == nullptr) return u32x4{0u, 0u, 0u, 0u};
    return load(sh, q % W);
  };
  u32x4 S[2 * W];  // P syndromes, then Q syndromes
#pragma unroll
  for (int s = 0; s < 2 * W; ++s) S[s] = u32x4{0u, 0u, 0u, 0u};
  u32x4 ring[RS];
#pragma unroll
  for (int q = 0; q < LA; ++q) ring[q] = fetch(q);
#pragma unroll
  for (int blk = 0; blk < W + 2; ++blk) {
    if (blk >= 2 && blk - 2 >= a.k) break;
    const int j = blk - 2;
    const int y = j > 0 ? (j * ((W - 1) / 2)) % W : 0;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const int p = blk * W + x, q = p + LA;
      if (q < NP) ring[q % RS] = fetch(q);
      const u32x4 v = ring[p % RS];
      if (blk < 2) {
        S[blk * W + x] ^= v;
      } else {
        S[x] ^= v;
        S[W + (x - j + W) % W] ^= v;
        if (j > 0 && x == (y + j - 1) % W) S[W + y] ^= v;
      }
    }
  }
  for (int b = 0; b < a.nout; ++b) {
    u32x4 acc[W];
#pragma unroll
    for (int x = 0; x < W; ++x) acc[x] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int s = 0; s < 2 * W; ++s) {
      const uint32_t bits = a.mbits[b][s];  // wave-uniform
      if (bits != 0u) {
#pragma unroll
        for (int x = 0; x < W; ++x) {
          const uint32_t m = (uint32_t)((int32_t)(bits << x) >> 31);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[x][e] ^= S[s][e] & m;
        }
      }
    }
    uint8_t* ob = const_cast<uint8_t*>(a.out[b].base) + o64 * a.out[b].stride;
    const uint32_t v = a.out[b].valid;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint32_t pk = (uint32_t)x * a.ps;
      if (full) st16<true>(ob + pk + off, acc[x]);
      else store_guarded(ob + pk, off, v > pk ? v - pk : 0u, acc[x]);
    }
  }
}

// ===========================================================================
// Liberation encode and decode with branch-free loads (round 5).
//
// lib_apply / lib_dec_apply above pick per load between a plain load (tile
// inside every shard) and load_guarded (a per-lane branch around the load).
// The uniform `full` test sits inside the unrolled packet loop, so every
// load sits between branches, and the compiler's wait-count pass then waits
// for ALL outstanding loads at each one: the shipped lib_apply<7> has 98
// loads and 79 `s_waitcnt vmcnt(0)` and no partial wait, so its "packets of
// look-ahead" never overlap (a wave has one 1 KiB load in flight at a time).
// Here the loads are raw buffer loads over one resource per block whose
// records end at the block's valid length rounded up to 16 (past it a load
// returns zeros without a memory access): no branch around any load, the
// look-ahead is real, and the wave-uniform `full` decision is taken once per
// tile, outside the loop (two copies of the body).  A tile that crosses a
// valid length clears the straddling chunk's tail where the packet is
// consumed (not where it is loaded, so its loads still overlap).  Absent
// shards (blocks past k, erased data blocks, coding blocks not in the
// survivor set) have base nullptr and valid 0: their loads return zeros.
__device__ __forceinline__ u32x4 libb_load(__amdgpu_buffer_rsrc_t rs, uint32_t vo) {
  return __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 2);  // nt
}
// An empty asm that "redefines" v: the XOR into v is done here, in ring
// order.  Without it the XORs of the straight-line body are reassociated into
// one tree at the end, so every loaded packet stays live (49 x 4 VGPRs at
// w = 7: the body spills).
__device__ __forceinline__ void libb_pin(u32x4& v) { asm volatile("" : "+v"(v)); }
// Bytes at or past `valid` of the 16-byte chunk at `pos` cleared.
__device__ __forceinline__ u32x4 libb_clip(u32x4 v, uint32_t valid, uint32_t pos) {
  const uint32_t n = valid > pos ? (valid - pos < 16u ? valid - pos : 16u) : 0u;
  return keep_first(v, n);
}

template <int W, int K, int LA, bool FULL>
__device__ __forceinline__ void libb_enc_tile(const LibArgs& a, uint64_t o64, uint32_t off,
                                              bool live) {
  constexpr int RS = LA + 1;  // ring of packet registers: LA loads in flight
  uint32_t vo[W];
#pragma unroll
  for (int x = 0; x < W; ++x) vo[x] = off + (uint32_t)x * a.ps;
  // block j's resource, built where it is used (SGPR arithmetic; an array
  // of resources is not promoted to registers at w >= 11)
  auto rs = [&](int j) {
    return shard_rsrc(a.in[j].base, a.in[j].stride, a.in[j].valid, o64, 16u);
  };
  u32x4 P[W], Q[W], ring[RS];
#pragma unroll
  for (int x = 0; x < W; ++x) P[x] = Q[x] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int q = 0; q < LA && q < K * W; ++q) ring[q] = libb_load(rs(q / W), vo[q % W]);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int y = (j * ((W - 1) / 2)) % W;  // Q row of block j's extra one
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const int p = j * W + x, q = p + LA;  // packet applied / packet loaded
      if (q < K * W) ring[q % RS] = libb_load(rs(q / W), vo[q % W]);
      u32x4 v = ring[p % RS];
      if (!FULL) v = libb_clip(v, a.in[j].valid, vo[x]);
      P[x] ^= v;
      Q[(x - j + W) % W] ^= v;
      libb_pin(P[x]);
      libb_pin(Q[(x - j + W) % W]);
      if (j > 0 && x == (y + j - 1) % W) {
        Q[y] ^= v;
        libb_pin(Q[y]);
      }
      // and the loads where the ring puts them (not hoisted further)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (!live) return;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint8_t* b = const_cast<uint8_t*>(a.out[r].base) + o64 * a.out[r].stride;
    const uint32_t v = a.out[r].valid;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const u32x4 acc = r == 0 ? P[x] : Q[x];
      if (FULL) st16<true>(b + vo[x], acc);
      else store_guarded(b, vo[x], v, acc);
    }
  }
}

template <int W, int K, int LA, int TW>
__global__ void __launch_bounds__(TW) __attribute__((amdgpu_waves_per_eu(lib_waves(W), 8)))
libb_apply(const LibArgs a) {
  constexpr uint32_t kTileBytes = TW * 16u;
  const uint32_t bid = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t t0 = tile * kTileBytes;
  const uint32_t off = t0 + threadIdx.x * 16u;
  // wave-uniform, as lib_apply's
  const bool full = t0 + kTileBytes <= a.ps &&
                    (uint64_t)(W - 1) * a.ps + t0 + kTileBytes <= (uint64_t)a.vmin;
  // lanes past the packet (last tile) load and compute but do not store
  if (full) libb_enc_tile<W, K, LA, true>(a, obj, off, true);
  else libb_enc_tile<W, K, LA, false>(a, obj, off, off < a.ps);
}

template <int W, int K, int LA, bool FULL>
__device__ __forceinline__ void libb_dec_tile(const LibDecArgs& a, uint64_t o64, uint32_t off,
                                              bool live) {
  constexpr int RS = LA + 1, NB = K + 2, NP = NB * W;  // LA = 0: the block form below
  uint32_t vo[W];
#pragma unroll
  for (int x = 0; x < W; ++x) vo[x] = off + (uint32_t)x * a.ps;
  // one packet stream: P (W packets), Q (W), then data blocks 0..k-1, as
  // lib_dec_apply; absent shards read as zeros through an empty resource
  auto shard_of = [&](int blk) -> const DevShard& {  // blk: 0 P, 1 Q, 2 + j data j
    return blk < 2 ? a.cod[blk] : a.data[blk - 2];
  };
  auto rs = [&](int b) {
    const DevShard& sh = shard_of(b);
    return shard_rsrc(sh.base, sh.stride, sh.valid, o64, 16u);
  };
  u32x4 S[2 * W];  // P syndromes, then Q syndromes
#pragma unroll
  for (int s = 0; s < 2 * W; ++s) S[s] = u32x4{0u, 0u, 0u, 0u};
  auto eat = [&](int blk, int x, u32x4 v) {  // packet x of stream block blk
    const int j = blk - 2;
    const int y = j > 0 ? (j * ((W - 1) / 2)) % W : 0;
    if (!FULL) v = libb_clip(v, shard_of(blk).valid, vo[x]);
    if (blk < 2) {
      S[blk * W + x] ^= v;
      libb_pin(S[blk * W + x]);
    } else {
      S[x] ^= v;
      S[W + (x - j + W) % W] ^= v;
      libb_pin(S[x]);
      libb_pin(S[W + (x - j + W) % W]);
      if (j > 0 && x == (y + j - 1) % W) {
        S[W + y] ^= v;
        libb_pin(S[W + y]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // as libb_enc_tile
  };
  if constexpr (LA == 0) {
    // block form: an absent shard (erased data block, coding block not a
    // survivor) is skipped by a uniform branch instead of streamed as zeros
    // (at k = 4 a third of the stream); a present block's w loads are in
    // flight together, then consumed
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) {
      if (shard_of(blk).base == nullptr) continue;
      const auto r = rs(blk);
      u32x4 yv[W];
#pragma unroll
      for (int x = 0; x < W; ++x) yv[x] = libb_load(r, vo[x]);
#pragma unroll
      for (int x = 0; x < W; ++x) eat(blk, x, yv[x]);
    }
  } else {
    u32x4 ring[RS];
#pragma unroll
    for (int q = 0; q < LA; ++q) ring[q] = libb_load(rs(q / W), vo[q % W]);
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) {
#pragma unroll
      for (int x = 0; x < W; ++x) {
        const int p = blk * W + x, q = p + LA;
        if (q < NP) ring[q % RS] = libb_load(rs(q / W), vo[q % W]);
        eat(blk, x, ring[p % RS]);
      }
    }
  }
  if (!live) return;
  // (unrolled over the <= 2 wanted blocks: as a run-time loop, the edge
  // path's byte-store addresses of both were hoisted out of it and spilled)
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    if (b >= a.nout) break;
    u32x4 acc[W];
#pragma unroll
    for (int x = 0; x < W; ++x) acc[x] = u32x4{0u, 0u, 0u, 0u};
    // (masked: an XOR only where a bit is set, behind uniform branches, read
    // 1-4 % slower, profiles/r06_s4_ab_lib*_combine.log)
#pragma unroll
    for (int s = 0; s < 2 * W; ++s) {
      const uint32_t bits = a.mbits[b][s];  // wave-uniform
      if (bits != 0u) {
#pragma unroll
        for (int x = 0; x < W; ++x) {
          const uint32_t m = (uint32_t)((int32_t)(bits << x) >> 31);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[x][e] ^= S[s][e] & m;
        }
      }
    }
    uint8_t* ob = const_cast<uint8_t*>(a.out[b].base) + o64 * a.out[b].stride;
    const uint32_t v = a.out[b].valid;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      if (FULL) st16<true>(ob + vo[x], acc[x]);
      else store_guarded(ob, vo[x], v, acc[x]);
    }
  }
}

template <int W, int K, int LA, int TW>
__global__ void __launch_bounds__(TW) __attribute__((amdgpu_waves_per_eu(lib_dec_waves(W), 8)))
libb_dec_apply(const LibDecArgs a) {
  constexpr uint32_t kTileBytes = TW * 16u;
  const uint32_t bid = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t t0 = tile * kTileBytes;
  const uint32_t off = t0 + threadIdx.x * 16u;
  const bool full = t0 + kTileBytes <= a.ps &&
                    (uint64_t)(W - 1) * a.ps + t0 + kTileBytes <= (uint64_t)a.vmin;
  if (full) libb_dec_tile<W, K, LA, true>(a, obj, off, true);
  else libb_dec_tile<W, K, LA, false>(a, obj, off, off < a.ps);
}

// Launch tables of libb_apply / libb_dec_apply, one translation unit per w
// (lib_inst.hip, every k = 1..w compiled in): the instance for (k, look-ahead
// la, tw lanes), or the shipped (la, tw) when that form is not built
// (measurement forms exist for the A/B configs only); fn nullptr for a w
// without instances.
using LibbEncFn = void (*)(const LibArgs);
using LibbDecFn = void (*)(const LibDecArgs);
struct LibbEnc {
  LibbEncFn fn;
  uint32_t lanes;
};
struct LibbDec {
  LibbDecFn fn;
  uint32_t lanes;
};
// The shipped liberation forms (round 5; interleaved A/B on two boxes,
// profiles/r05_s3_ab_lib_*.log, r05_s4_ab_lib_*.log):
//  encode: libb_apply (look-ahead 2, 64 lanes) for w >= 11 (+1 to +6 %);
//          lib_apply below (libb_apply -2 to -8 % at w <= 7);
//  decode and repair through syndromes: libb_dec_apply with 64 lanes,
//          look-ahead 4 at w = 13 or k <= 4, 2 otherwise (+5 to +16 % at
//          w >= 7 with k >= 7, +2 % at (4,2,7) with look-ahead 4, within
//          +-4 % at (5,2,5)).
constexpr int kLibbEncLA = 2, kLibbEncTW = 64, kLibbEncMinW = 11;
constexpr int kLibbDecTW = 64;
constexpr int libb_dec_la(int w, int k) { return (w >= 13 || k <= 4) ? 4 : 2; }
template <int W>
LibbEnc libb_enc_pick(int k, int la, int tw);
template <int W>
LibbDec libb_dec_pick(int k, int la, int tw);

// ===========================================================================
// GF(2^w) on packet-bitsliced blocks (cauchyrs).  Each lane owns LW dwords of
// every packet.  Per input block: y = its w packets; for t = 0..w-1, every
// output block whose coefficient has bit t set gets y xor-ed in, then
// y <- y * 2 in bitsliced form (a rename plus one xor per set low bit of the
// primitive polynomial).  Cost per packet dword ~ popcount(coef) + 3, against
// m*w masked xors for a generic bitmatrix.
template <int R>
struct GfbArgs {
  DevShard in[kMaxK];
  DevShard out[R];
  uint32_t coef[R][kMaxK];
  int K;
  uint32_t ps;     // packet bytes
  uint32_t tiles;  // tiles per object (over one packet)
  uint32_t xmap;   // 1: xcd_obj_map
};

template <int W>
struct DefaultPoly;  // low bits of the gf-complete default polynomial
template <> struct DefaultPoly<2> { static constexpr uint32_t v = 03; };
template <> struct DefaultPoly<3> { static constexpr uint32_t v = 03; };
template <> struct DefaultPoly<4> { static constexpr uint32_t v = 03; };
template <> struct DefaultPoly<5> { static constexpr uint32_t v = 05; };
template <> struct DefaultPoly<6> { static constexpr uint32_t v = 03; };
template <> struct DefaultPoly<7> { static constexpr uint32_t v = 011; };
template <> struct DefaultPoly<8> { static constexpr uint32_t v = 035; };
template <> struct DefaultPoly<9> { static constexpr uint32_t v = 021; };
template <> struct DefaultPoly<10> { static constexpr uint32_t v = 011; };
template <> struct DefaultPoly<11> { static constexpr uint32_t v = 05; };
template <> struct DefaultPoly<12> { static constexpr uint32_t v = 0123; };
template <> struct DefaultPoly<13> { static constexpr uint32_t v = 033; };
template <> struct DefaultPoly<14> { static constexpr uint32_t v = 02103; };
template <> struct DefaultPoly<15> { static constexpr uint32_t v = 03; };
template <> struct DefaultPoly<16> { static constexpr uint32_t v = 010013; };

template <int LW>
struct LaneVec {
  uint32_t v[LW];
};

template <int LW>
__device__ __forceinline__ LaneVec<LW> lv_load(const uint8_t* p, uint32_t off, uint32_t valid) {
  LaneVec<LW> r;
  if (LW == 4) {
    const u32x4 x = load_guarded(p, off, valid);
#pragma unroll
    for (int e = 0; e < 4; ++e) r.v[e] = x[e];
  } else {
    typedef uint32_t vt __attribute__((ext_vector_type(LW == 1 ? 1 : 2)));
    const uint32_t bytes = 4u * LW;
    if (off + bytes <= valid) {
      if (LW == 2) {
        const vt x = __builtin_nontemporal_load(reinterpret_cast<const vt*>(p + off));
        r.v[0] = x[0];
        r.v[LW - 1] = x[LW == 2 ? 1 : 0];
      } else {
        r.v[0] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p + off));
      }
    } else {
#pragma unroll
      for (int e = 0; e < LW; ++e) {
        const uint32_t o = off + 4u * e;
        uint32_t w = 0;
        if (o < valid) {
          w = *reinterpret_cast<const uint32_t*>(p + o);
          const uint32_t n = valid - o;
          if (n < 4) w &= (1u << (8u * n)) - 1u;
        }
        r.v[e] = w;
      }
    }
  }
  return r;
}

template <int LW>
__device__ __forceinline__ void lv_store(uint8_t* p, uint32_t off, uint32_t valid,
                                         const LaneVec<LW>& x) {
  const uint32_t bytes = 4u * LW;
  if (off + bytes <= valid) {
    if (LW == 4) {
      st16<true>(p + off, u32x4{x.v[0], x.v[1 % LW], x.v[2 % LW], x.v[3 % LW]});
    } else if (LW == 2) {
      typedef uint32_t v2 __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(v2{x.v[0], x.v[LW - 1]}, reinterpret_cast<v2*>(p + off));
    } else {
      __builtin_nontemporal_store(x.v[0], reinterpret_cast<uint32_t*>(p + off));
    }
  } else if (off < valid) {
    const uint32_t n = valid - off;
#pragma unroll
    for (int i = 0; i < 4 * LW; ++i)
      if ((uint32_t)i < n) p[off + i] = (uint8_t)(x.v[i >> 2] >> (8 * (i & 3)));
  }
}

template <int W, int LW>
__device__ __forceinline__ void gfb_load_block(const uint8_t* base, uint32_t ps, uint32_t off,
                                               uint32_t bv, LaneVec<LW> (&y)[W]) {
#pragma unroll
  for (int x = 0; x < W; ++x) y[x] = lv_load<LW>(base + (uint32_t)x * ps, off, packet_valid(bv, x, ps));
}

// acc[i] ^= c[i] * y for every output i (y is consumed: it is doubled in
// place).  CEIL (measurement only): every input xor-ed into every output, no
// GF arithmetic — the memory ceiling of the access pattern, not a code.
template <int W, int R, int LW, bool CEIL>
__device__ __forceinline__ void gfb_accumulate(LaneVec<LW> (&acc)[R][W], LaneVec<LW> (&y)[W],
                                               const uint32_t (&c)[R]) {
  if (CEIL) {
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int x = 0; x < W; ++x)
#pragma unroll
        for (int e = 0; e < LW; ++e) acc[i][x].v[e] ^= y[x].v[e];
    return;
  }
#pragma unroll
  for (int t = 0; t < W; ++t) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if ((c[i] >> t) & 1u) {
#pragma unroll
        for (int x = 0; x < W; ++x)
#pragma unroll
          for (int e = 0; e < LW; ++e) acc[i][x].v[e] ^= y[x].v[e];
      }
    }
    if (t + 1 < W) {  // y <- y * 2
      const LaneVec<LW> top = y[W - 1];
#pragma unroll
      for (int r = W - 1; r >= 1; --r) {
#pragma unroll
        for (int e = 0; e < LW; ++e)
          y[r].v[e] = ((DefaultPoly<W>::v >> r) & 1u) ? (y[r - 1].v[e] ^ top.v[e]) : y[r - 1].v[e];
      }
      y[0] = top;
    }
  }
}

// Input staging forms:
//   KR > 0 : all (<= KR) input blocks are loaded before any arithmetic, so a
//            wave has every load of its tile in flight at once (like gf8);
//   PFD > 0: the loads of the next PFD blocks are in flight while block j is
//            computed (a ring of PFD+1 blocks in VGPRs);
//   PFD = 0: load block j, then compute on it.
//   WAVES > 0: ask the register allocator for at least WAVES waves per SIMD
//            (amdgpu_waves_per_eu; 4 caps the kernel at 128 VGPRs).
template <int W, int R, int LW, bool ACC, int PFD = 1, bool CEIL = false, int KR = 0,
          int WG = kThreads, int XMAP = 0, int WAVES = 0>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(WAVES > 0 ? WAVES : 1, 8)))
gfbit_apply(const GfbArgs<R> a) {
  constexpr uint32_t LB = 4u * LW;
  const uint32_t bid = XMAP == 1 ? xcd_group(blockIdx.x, gridDim.x)
                       : (XMAP == 2 || a.xmap) ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles)
                                               : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t off = packet_lane_off(tile, threadIdx.x, WG, LB);
  if (off >= a.ps) return;
  const uint64_t o64 = obj;
  LaneVec<LW> acc[R][W];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int x = 0; x < W; ++x) {
      if (ACC) {
        const uint32_t pk = (uint32_t)x * a.ps;
        acc[i][x] = lv_load<LW>(a.out[i].base + o64 * a.out[i].stride + pk, off,
                                packet_valid(a.out[i].valid, x, a.ps));
      } else {
#pragma unroll
        for (int e = 0; e < LW; ++e) acc[i][x].v[e] = 0u;
      }
    }
  auto coefs = [&](int j, uint32_t (&c)[R]) {
#pragma unroll
    for (int i = 0; i < R; ++i) c[i] = a.coef[i][j];
  };
  auto load = [&](int j, LaneVec<LW> (&y)[W]) {
    gfb_load_block<W, LW>(a.in[j].base + o64 * a.in[j].stride, a.ps, off, a.in[j].valid, y);
  };
  if constexpr (KR > 0) {
    LaneVec<LW> ys[KR][W];
#pragma unroll
    for (int j = 0; j < KR; ++j)
      if (j < a.K) load(j, ys[j]);
#pragma unroll
    for (int j = 0; j < KR; ++j) {
      if (j < a.K) {
        uint32_t c[R];
        coefs(j, c);
        gfb_accumulate<W, R, LW, CEIL>(acc, ys[j], c);
      }
    }
  } else {
    constexpr int RS = PFD + 1;
    LaneVec<LW> ring[RS][W];
#pragma unroll
    for (int u = 0; u < PFD; ++u)
      if (u < a.K) load(u, ring[u]);
    for (int j0 = 0; j0 < a.K; j0 += RS) {
#pragma unroll
      for (int u = 0; u < RS; ++u) {
        const int j = j0 + u;
        if (j < a.K) {
          if (j + PFD < a.K) load(j + PFD, ring[(u + PFD) % RS]);
          uint32_t c[R];
          coefs(j, c);
          gfb_accumulate<W, R, LW, CEIL>(acc, ring[u], c);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    uint8_t* p = const_cast<uint8_t*>(a.out[i].base) + o64 * a.out[i].stride;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint32_t pk = (uint32_t)x * a.ps;
      lv_store<LW>(p + pk, off, packet_valid(a.out[i].valid, x, a.ps), acc[i][x]);
    }
  }
}

// ===========================================================================
// Host-side launch templates.
inline DevShard dev_shard(const Shard& s, uint64_t o0) {
  DevShard d;
  d.base = s.base + o0 * s.stride;
  d.stride = s.stride;
  d.valid = (uint32_t)s.valid;
  d.pad = 0;
  return d;
}

inline uint32_t gf8_mul_host(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (; b; b >>= 1) {
    if (b & 1) r ^= a;
    a <<= 1;
    if (a & 0x100) a ^= 0x11D;
  }
  return r;
}

// v_perm tables (T0 lo, T0 hi, T1 lo, T1 hi, T2) for multiply-by-c in GF(2^8).
inline void gf8_tables(uint32_t c, uint32_t t[5]) {
  uint8_t b0[8], b1[8], b2[4];
  for (int i = 0; i < 8; ++i) {
    b0[i] = (uint8_t)gf8_mul_host(c, (uint32_t)i);
    b1[i] = (uint8_t)gf8_mul_host(c, (uint32_t)(i << 3));
  }
  for (int i = 0; i < 4; ++i) b2[i] = (uint8_t)gf8_mul_host(c, (uint32_t)(i << 6));
  auto pack = [](const uint8_t* b) {
    return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
  };
  t[0] = pack(b0);
  t[1] = pack(b0 + 4);
  t[2] = pack(b1);
  t[3] = pack(b1 + 4);
  t[4] = pack(b2);
}

int device_cus();         // compute units of the current device (kernels.hip)
int gf8_tile_map();       // gf8_apply workgroup -> tile order (kernels.hip)
int gf8_wg_env();         // LEOEC_GF8_WG override of the tile width (kernels.hip)
bool gf8_tile_map_set();  // LEOEC_GF8_TMAP given (then no automatic xcd_obj_map)
int gf8_tile_group();     // tiles per XCD group of tile map 4 (kernels.hip)
// Blocks larger than this run gf8_apply with 64-lane workgroups: 1 MiB objects
// (bs 104,960) keep 256 lanes, 2 MiB (209,792) and up take 64.
constexpr uint64_t kGf8NarrowBytes = 160 * 1024;

// BRANCHY = -1: pick per launch from the coefficients (scalar-branch form
// when enough coefficients are 0/1, the paired all-table form otherwise).
template <int K, int R, bool ACC, int CPT = kGf8Default.cpt, bool NT = kGf8Default.nt,
          int BRANCHY = kGf8Default.branchy, bool COPY = kGf8Default.copy, bool PIPE = false,
          bool LDS = kGf8Default.lds, int WAVES = kGf8Default.waves, int WG = kThreads,
          int XMAP = kGf8Default.xmap, bool BUF = false, bool ONES = false, bool EARLY = false>
int launch_gf8_t(const GfApply& p, const Chunk& c, hipStream_t s) {
  Gf8Args<K, R> a;
  a.one = a.zero = 0;
  uint32_t vmin = 0xFFFFFFFFu;
  int n01 = 0;
  for (int j = 0; j < K; ++j) {
    a.in[j] = dev_shard(p.in[c.j0 + j], c.o0);
    vmin = a.in[j].valid < vmin ? a.in[j].valid : vmin;
  }
  for (int r = 0; r < R; ++r) {
    a.out[r] = dev_shard(p.out[c.r0 + r], c.o0);
    vmin = a.out[r].valid < vmin ? a.out[r].valid : vmin;
    for (int j = 0; j < K; ++j) {
      const uint32_t cf = p.coef[(size_t)(c.r0 + r) * p.K + c.j0 + j] & 0xFFu;
      gf8_tables(cf, a.tab[r][j]);
      if (cf == 1) a.one |= 1ull << (r * K + j);
      if (cf == 0) a.zero |= 1ull << (r * K + j);
      n01 += cf <= 1;
    }
  }
  // Workgroup (= tile) width: WG lanes, or 64 lanes (1 KiB tiles) for blocks
  // above kGf8NarrowBytes, where they measured 2-8 % faster (block
  // size sweep); LEOEC_GF8_WG=64|256 forces one (A/B, parity tests).
  uint32_t wg = (uint32_t)WG;
  if (CPT == 1 && !PIPE) {
    const int force = gf8_wg_env();
    if (force == 64 || (force == 0 && p.block_size > kGf8NarrowBytes)) wg = 64;
  }
  const uint32_t tb = wg * 16u * CPT;
  a.tiles = (uint32_t)((p.block_size + tb - 1) / tb);
  a.vmin = vmin;
  a.total_tiles = (uint32_t)(c.no * a.tiles);
  a.nobj = (uint32_t)c.no;
  a.tmap = (uint32_t)gf8_tile_map();
  a.tperm = 1;
  if (a.tmap == 0 && !gf8_tile_map_set()) {  // shipped choice (measure build: unless forced)
    if (a.tiles <= kObjMapMaxTiles) {
      a.tmap = 3;
    } else if (a.tiles >= kSegMapMinTiles) {
      a.tmap = 4;
      a.tperm = kSegMapGroup;
    }
  }
  if (a.tmap == 4 && gf8_tile_group() > 0) a.tperm = (uint32_t)gf8_tile_group();
  if (a.tmap == 2) {  // stride ~ tiles / 16, coprime with tiles (a bijection on tiles)
    uint32_t q = a.tiles / 16u + 1u;
    auto gcd = [](uint32_t x, uint32_t y) { while (y) { const uint32_t t = x % y; x = y; y = t; } return x; };
    while (gcd(q, a.tiles) != 1u) ++q;
    a.tperm = q % a.tiles ? q % a.tiles : 1u;
  }
  // per-dword VALU: general coefficient 5.5 (branchy) vs 5 (paired); a 1 costs
  // 1 and a 0 nothing in the branchy form
  const int n = R * K;
  const bool branchy = BRANCHY >= 0 ? BRANCHY != 0 : (11 * (n - n01) + 2 * n01 < 10 * n);
  uint32_t grid = a.total_tiles;
  if (PIPE) {
    const uint32_t cap = (uint32_t)device_cus() * 4u;
    grid = grid < cap ? grid : cap;
  }
  // ONES: row 0 and column 0 of this launch's coefficients are all 1
  bool ones = ONES && c.r0 == 0 && c.j0 == 0;
  for (int r = 0; ones && r < R; ++r)
    for (int j = 0; ones && j < K; ++j)
      if ((r == 0 || j == 0) && (p.coef[(size_t)r * p.K + j] & 0xFFu) != 1u) ones = false;
  if (ONES && ones) {
    hipLaunchKernelGGL((gf8_apply<K, R, ACC, CPT, NT, false, COPY, PIPE, LDS, WAVES, WG, XMAP, BUF, true, EARLY>),
                       dim3(grid), dim3(wg), 0, s, a);
    return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
  }
  if (branchy)
    hipLaunchKernelGGL((gf8_apply<K, R, ACC, CPT, NT, true, COPY, PIPE, LDS, WAVES, WG, XMAP, BUF, false, EARLY>),
                       dim3(grid), dim3(wg), 0, s, a);
  else
    hipLaunchKernelGGL((gf8_apply<K, R, ACC, CPT, NT, false, COPY, PIPE, LDS, WAVES, WG, XMAP, BUF, false, EARLY>),
                       dim3(grid), dim3(wg), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

using ChunkFn = int (*)(const GfApply&, const Chunk&, hipStream_t);

// Defined (explicitly instantiated) in gf8_inst.hip, one TU per K.
template <int K>
ChunkFn gf8_launcher(int r, bool acc);

// Measurement variants of gf8_apply<10, 4> (gf8_exp.hip); nullptr if unknown.
// gf8_variant_part<P> holds the variants n with n % 4 == P (one TU each).
ChunkFn gf8_variant(int variant);
template <int P>
ChunkFn gf8_variant_part(int variant);

// Bitsliced GF(2^16) / GF(2^32) launches (gfs_inst.hip), r = 1..kMaxR outputs.
ChunkFn gfs_pick(int w, int r, bool acc);

}  // namespace detail
}  // namespace leoec

#ifdef LEOEC_MEASURE
// The measurement build's superseded kernel forms (A/B and parity only).
#include "kernels_measure.hpp"
#endif
