// kernels_measure.hpp — kernel forms of the MEASUREMENT build only
// (libleoec_measure.so, -DLEOEC_MEASURE): the round-1 w = 16 / 32 kernels
// that the bitsliced gfs_apply (gfs_inst.hip) replaced — shift-and-add
// (gfw_apply), 2-bit-field v_perm (gf16_apply), byte planes (gfp_apply) —
// and the LDS-staged form of the cauchyrs packet kernel (gfbit_lds_apply).
// They stay parity-tested A/B references (tests/test_gpu_parity.py
// test_gfw_kernel_forms_agree / test_cauchy_kernel_forms_agree); the
// product library never compiles them.  Included at the end of
// kernels_impl.hpp.
#pragma once

#ifndef LEOEC_MEASURE
#error "measurement build only"
#endif

namespace leoec {
namespace detail {

// ===========================================================================
// GF(2^16) / GF(2^32): shift-and-add over little-endian words, K runtime.
template <int R>
struct GfwArgs {
  DevShard in[kMaxK];
  DevShard out[R];
  uint32_t coef[R][kMaxK];
  int K;
  uint32_t tiles;
  uint32_t vmin;
};

template <int W>
__device__ __forceinline__ uint32_t xtime(uint32_t x) {
  if (W == 32) {  // x^32 = x^22 + x^2 + x + 1
    const uint32_t sign = (uint32_t)((int32_t)x >> 31);
    return (x << 1) ^ (sign & 0x00400007u);
  } else {  // two packed 16-bit words, x^16 = x^12 + x^3 + x + 1
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    const u16x2 v = __builtin_bit_cast(u16x2, x);
    const u16x2 sh = v << (unsigned short)1;
    const s16x2 sg = __builtin_bit_cast(s16x2, v) >> (short)15;
    return __builtin_bit_cast(uint32_t, sh) ^ (__builtin_bit_cast(uint32_t, sg) & 0x100B100Bu);
  }
}

template <int W, int R, bool ACC>
__global__ void __launch_bounds__(kThreads) gfw_apply(const GfwArgs<R> a) {
  const uint32_t obj = blockIdx.x / a.tiles;
  const uint32_t tile = blockIdx.x - obj * a.tiles;
  const uint32_t t0 = tile * kTileBytes;
  const uint32_t off = t0 + threadIdx.x * 16u;
  const bool full = t0 + kTileBytes <= a.vmin;
  const uint64_t o = obj;
  u32x4 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    acc[r] = u32x4{0u, 0u, 0u, 0u};
    if (ACC) acc[r] = load_guarded(a.out[r].base + o * a.out[r].stride, off, a.out[r].valid);
  }
  for (int j = 0; j < a.K; ++j) {
    const uint8_t* p = a.in[j].base + o * a.in[j].stride;
    u32x4 x = full ? ld16<true>(p + off) : load_guarded(p, off, a.in[j].valid);
    uint32_t c[R];
#pragma unroll
    for (int r = 0; r < R; ++r) c[r] = a.coef[r][j];
#pragma unroll
    for (int b = 0; b < W; ++b) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t m = (uint32_t)(-(int32_t)((c[r] >> b) & 1u));
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[r][e] ^= x[e] & m;
      }
      if (b + 1 < W) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = xtime<W>(x[e]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
    store_guarded(const_cast<uint8_t*>(a.out[r].base) + o * a.out[r].stride, off, a.out[r].valid,
                  acc[r]);
}

// ===========================================================================
// GF(2^16) with v_perm over 2-bit fields.  A dword holds two little-endian
// words; for field f (bits 2f, 2f+1 of each word) one v_perm returns both
// 16-bit products c*(v << 2f) at once: selector bytes [v0, v0|4, v1, v1|4]
// pick the low byte of the product from a 4-entry table in src1 and the
// high byte from one in src0.  8 perms + 4 xor3 per coefficient per dword;
// the 8 selector dwords of an input dword are shared by every row.  Tables
// (R x K coefficients x 8 fields x 2 dwords) are built in LDS by the block.
template <int R>
struct Gf16Args {
  DevShard in[kMaxK];
  DevShard out[R];
  uint32_t coef[R][kMaxK];
  int K;
  uint32_t tiles;
  uint32_t vmin;
};

__device__ __forceinline__ uint32_t gf16_x2(uint32_t v) {  // v * x mod 0x1100B
  return ((v << 1) ^ ((v & 0x8000u) ? 0x1100Bu : 0u)) & 0xFFFFu;
}

template <int R, bool ACC>
__global__ void __launch_bounds__(kThreads) gf16_apply(const Gf16Args<R> a) {
  __shared__ uint32_t tab[R * kMaxK][8][2];
  const int K = a.K;
  for (int i = threadIdx.x; i < R * K * 8; i += kThreads) {
    const int ci = i >> 3, f = i & 7;
    uint32_t d1 = a.coef[ci / K][ci % K] & 0xFFFFu;
    for (int t = 0; t < 2 * f; ++t) d1 = gf16_x2(d1);
    const uint32_t d2 = gf16_x2(d1), d3 = d1 ^ d2;
    tab[ci][f][0] = ((d1 & 0xFFu) << 8) | ((d2 & 0xFFu) << 16) | ((d3 & 0xFFu) << 24);
    tab[ci][f][1] = ((d1 >> 8) << 8) | ((d2 >> 8) << 16) | ((d3 >> 8) << 24);
  }
  __syncthreads();
  const uint32_t obj = blockIdx.x / a.tiles;
  const uint32_t tile = blockIdx.x - obj * a.tiles;
  const uint32_t t0 = tile * kTileBytes;
  const uint32_t off = t0 + threadIdx.x * 16u;
  const bool full = t0 + kTileBytes <= a.vmin;
  const uint64_t o = obj;
  u32x4 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    acc[r] = u32x4{0u, 0u, 0u, 0u};
    if (ACC) acc[r] = load_guarded(a.out[r].base + o * a.out[r].stride, off, a.out[r].valid);
  }
  for (int j = 0; j < K; ++j) {
    const uint8_t* p = a.in[j].base + o * a.in[j].stride;
    const u32x4 x = full ? ld16<true>(p + off) : load_guarded(p, off, a.in[j].valid);
    uint32_t sel[8][4];
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t t = (x[e] >> (2 * f)) & 0x00030003u;
        sel[f][e] = (t << 8) | t | 0x04000400u;
      }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t(*tb)[2] = tab[r * K + j];
#pragma unroll
      for (int f = 0; f < 8; f += 2) {
        const uint32_t l0 = tb[f][0], h0 = tb[f][1], l1 = tb[f + 1][0], h1 = tb[f + 1][1];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[r][e] = xor3(acc[r][e], perm(h0, l0, sel[f][e]), perm(h1, l1, sel[f + 1][e]));
      }
    }
  }
  if (full) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      st16<true>(const_cast<uint8_t*>(a.out[r].base) + o * a.out[r].stride + off, acc[r]);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
      store_guarded(const_cast<uint8_t*>(a.out[r].base) + o * a.out[r].stride, off,
                    a.out[r].valid, acc[r]);
  }
}

// ===========================================================================
// GF(2^16) / GF(2^32) on byte planes.  Multiplication by c is GF(2)-linear,
// so byte o of c*x is the XOR over input bytes b of M_ob(x_b), with M_ob(v) =
// byte o of c*(v << 8b): an 8-bit -> 8-bit linear map, applied exactly like
// the GF(2^8) kernel applies a coefficient (three v_perm lookups of 8-entry
// byte tables over the 3/3/2-bit split of v).  A v_perm applies one table to
// the four bytes of a dword, so a lane's 16-byte column is first transposed
// into byte planes: plane dword pd = b*G + g holds byte b of four words (G =
// 4 / NB dwords per plane, NB = W / 8 bytes per word).  Per coefficient and
// 4 words: NB*NB maps x 3 perms (w=32: 48 perms + 24 xor3; w=16, 8 words:
// 24 perms + 12 xor3), against 8*W masked xors + doublings for shift-and-add.
// Coefficients 1 / 0 take a scalar branch (plain xor / skip).  The per-
// coefficient tables are built in LDS by each workgroup (powers c*x^u, then
// the table bytes); the grid walks the tiles (grid-stride) so that prologue
// is paid a few times per CU, not once per tile.
template <int R>
struct GfpArgs {
  DevShard in[kMaxK];
  DevShard out[R];
  uint32_t coef[R][kMaxK];
  int K;
  uint32_t tiles;        // tiles per object
  uint32_t vmin;         // min valid over all shards of the launch
  uint32_t total_tiles;  // tiles of the launch
};

template <int W, int R>
struct GfpLds {
  static constexpr int NB = W / 8, NM = NB * NB, N2 = (NM + 3) / 4;
  u32x4 t01[R * kMaxK][NM];  // map m = o*NB + b: T0 lo, T0 hi, T1 lo, T1 hi
  uint32_t t2[R * kMaxK][N2 * 4];  // T2 of map m at [m]
  uint32_t pw[R * kMaxK][W];       // c * x^u
};

template <int W>
__device__ __forceinline__ uint32_t gfw_xtime1(uint32_t v) {
  if (W == 32) return (v << 1) ^ ((v >> 31) ? 0x00400007u : 0u);
  return ((v << 1) ^ ((v & 0x8000u) ? 0x1100Bu : 0u)) & 0xFFFFu;
}

// Byte-plane transposes of one 16-byte column (self-inverse for W = 32).
template <int W>
__device__ __forceinline__ u32x4 to_planes(u32x4 x) {
  if (W == 32) {
    const uint32_t a0 = perm(x[1], x[0], 0x05010400u), a1 = perm(x[1], x[0], 0x07030602u);
    const uint32_t b0 = perm(x[3], x[2], 0x05010400u), b1 = perm(x[3], x[2], 0x07030602u);
    return u32x4{perm(b0, a0, 0x05040100u), perm(b0, a0, 0x07060302u), perm(b1, a1, 0x05040100u),
                 perm(b1, a1, 0x07060302u)};
  }
  // W = 16: [lo g0, lo g1, hi g0, hi g1], group g = words 4g..4g+3
  return u32x4{perm(x[1], x[0], 0x06040200u), perm(x[3], x[2], 0x06040200u),
               perm(x[1], x[0], 0x07050301u), perm(x[3], x[2], 0x07050301u)};
}
template <int W>
__device__ __forceinline__ u32x4 from_planes(u32x4 p) {
  if (W == 32) return to_planes<32>(p);
  return u32x4{perm(p[2], p[0], 0x05010400u), perm(p[2], p[0], 0x07030602u),
               perm(p[3], p[1], 0x05010400u), perm(p[3], p[1], 0x07030602u)};
}

template <int W, int R, bool ACC, int CPT>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 8)))
gfp_apply(const GfpArgs<R> a) {
  constexpr int NB = W / 8, G = 4 / NB;
  constexpr int NM = NB * NB;
  constexpr uint32_t CS = kTileBytes;
  constexpr uint32_t TB = CS * CPT;
  __shared__ GfpLds<W, R> L;
  const int K = a.K;
  const int nco = R * K;
  // prologue 1: powers c * x^u (one thread per coefficient, W serial steps)
  for (int ci = threadIdx.x; ci < nco; ci += kThreads) {
    uint32_t v = a.coef[ci / K][ci % K];
    for (int u = 0; u < W; ++u) {
      L.pw[ci][u] = v;
      v = gfw_xtime1<W>(v);
    }
  }
  __syncthreads();
  // prologue 2: the 20 table bytes of every (coefficient, map)
  for (int i = threadIdx.x; i < nco * NM; i += kThreads) {
    const int ci = i / NM, m = i - ci * NM;
    const int o = m / NB, b = m - o * NB;
    const uint32_t* pw = &L.pw[ci][8 * b];
    auto entry = [&](int t0, uint32_t v) {  // byte o of c * ((v << t0) << 8b)
      uint32_t s = 0;
      for (int t = 0; t < 3; ++t)
        if ((v >> t) & 1u) s ^= pw[t0 + t];
      return (s >> (8 * o)) & 0xFFu;
    };
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0;
    for (int e = 0; e < 4; ++e) {
      w0 |= entry(0, e) << (8 * e);
      w1 |= entry(0, e + 4) << (8 * e);
      w2 |= entry(3, e) << (8 * e);
      w3 |= entry(3, e + 4) << (8 * e);
      w4 |= entry(6, e) << (8 * e);
    }
    L.t01[ci][m] = u32x4{w0, w1, w2, w3};
    L.t2[ci][m] = w4;
  }
  __syncthreads();

  for (uint32_t g = blockIdx.x; g < a.total_tiles; g += gridDim.x) {
    const uint32_t obj = g / a.tiles;
    const uint32_t t0 = (g - obj * a.tiles) * TB;
    const uint32_t off = t0 + threadIdx.x * 16u;
    const bool full = t0 + TB <= a.vmin;  // wave-uniform
    const uint64_t o64 = obj;
    u32x4 acc[R][CPT];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        acc[r][c] = u32x4{0u, 0u, 0u, 0u};
        if (ACC)
          acc[r][c] = to_planes<W>(
              load_guarded(a.out[r].base + o64 * a.out[r].stride, off + c * CS, a.out[r].valid));
      }
    auto load = [&](int j, u32x4 (&x)[CPT]) {
      const uint8_t* p = a.in[j].base + o64 * a.in[j].stride;
#pragma unroll
      for (int c = 0; c < CPT; ++c)
        x[c] = full ? ld16<true>(p + off + c * CS) : load_guarded(p, off + c * CS, a.in[j].valid);
    };
    u32x4 nxt[CPT];
    load(0, nxt);
    for (int j = 0; j < K; ++j) {
      u32x4 pl[CPT];
#pragma unroll
      for (int c = 0; c < CPT; ++c) pl[c] = to_planes<W>(nxt[c]);
      if (j + 1 < K) load(j + 1, nxt);
      uint32_t s0[CPT][4], s1[CPT][4], s2[CPT][4];
#pragma unroll
      for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          s0[c][d] = pl[c][d] & 0x07070707u;
          s1[c][d] = (pl[c][d] >> 3) & 0x07070707u;
          s2[c][d] = (pl[c][d] >> 6) & 0x03030303u;
        }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t cf = a.coef[r][j];  // wave-uniform
        if (cf == 0u) continue;
        if (cf == 1u) {
#pragma unroll
          for (int c = 0; c < CPT; ++c) acc[r][c] ^= pl[c];
          continue;
        }
        const int ci = r * K + j;
#pragma unroll
        for (int o = 0; o < NB; ++o) {
          u32x4 t[NB];
          uint32_t t2[NB];
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            t[b] = L.t01[ci][o * NB + b];
            t2[b] = L.t2[ci][o * NB + b];
          }
#pragma unroll
          for (int gg = 0; gg < G; ++gg)
#pragma unroll
            for (int c = 0; c < CPT; ++c) {
              uint32_t p[3 * NB];  // 3*NB terms (even), folded pairwise into acc by xor3
#pragma unroll
              for (int b = 0; b < NB; ++b) {
                const int d = b * G + gg;
                p[3 * b] = perm(t[b][1], t[b][0], s0[c][d]);
                p[3 * b + 1] = perm(t[b][3], t[b][2], s1[c][d]);
                p[3 * b + 2] = perm(t2[b], t2[b], s2[c][d]);
              }
              uint32_t v = acc[r][c][o * G + gg];
#pragma unroll
              for (int q = 0; q < 3 * NB; q += 2) v = xor3(v, p[q], p[q + 1]);
              acc[r][c][o * G + gg] = v;
            }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      uint8_t* p = const_cast<uint8_t*>(a.out[r].base) + o64 * a.out[r].stride;
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const u32x4 v = from_planes<W>(acc[r][c]);
        if (full) st16<true>(p + off + c * CS, v);
        else store_guarded(p, off + c * CS, a.out[r].valid, v);
      }
    }
  }
}

// LDS-staged form of gfbit_apply.  The workgroup stages each input block's
// W packet slices (2 KiB each) through LDS: wave v loads half-packets, so a
// wave streams ceil(W/2) packets of 1 KiB contiguous per block instead of W
// packets of 512 B, and block j+1's loads are in flight (in VGPRs) while
// block j is computed from LDS.  Lanes then read their 8-byte columns of all
// W packets from LDS (conflict-free ds_read_b64) and run the same bitsliced
// arithmetic.  Outputs are stored directly.
constexpr int kGfbLdsThreads = 256;
constexpr uint32_t kGfbLdsSlice = kGfbLdsThreads * 8u;  // bytes per packet per tile

template <int W, int R, bool ACC>
__global__ void __launch_bounds__(kGfbLdsThreads) gfbit_lds_apply(const GfbArgs<R> a) {
  constexpr int LW = 2;
  constexpr int kChunks = W * (int)(kGfbLdsSlice / 16u);          // 16-B chunks per block
  constexpr int NQ = (kChunks + kGfbLdsThreads - 1) / kGfbLdsThreads;
  __shared__ u32x4 buf[2][kChunks];
  const uint32_t tid = threadIdx.x;
  const uint32_t obj = blockIdx.x / a.tiles;
  const uint32_t tile = blockIdx.x - obj * a.tiles;
  const uint32_t t0 = tile * kGfbLdsSlice;
  const uint32_t off = t0 + tid * 8u;
  const bool active = off < a.ps;
  const uint64_t o64 = obj;
  LaneVec<LW> acc[R][W];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int x = 0; x < W; ++x) {
      if (ACC && active) {
        const uint32_t pk = (uint32_t)x * a.ps;
        const uint32_t bv = a.out[i].valid;
        acc[i][x] = lv_load<LW>(a.out[i].base + o64 * a.out[i].stride + pk, off,
                                bv > pk ? bv - pk : 0u);
      } else {
#pragma unroll
        for (int e = 0; e < LW; ++e) acc[i][x].v[e] = 0u;
      }
    }
  u32x4 stage[NQ];
  auto gload = [&](int j) {
    const uint8_t* base = a.in[j].base + o64 * a.in[j].stride;
    const uint32_t bv = a.in[j].valid;
#pragma unroll
    for (int r = 0; r < NQ; ++r) {
      const uint32_t q = tid + (uint32_t)r * kGfbLdsThreads;
      stage[r] = u32x4{0u, 0u, 0u, 0u};
      if (q < (uint32_t)kChunks) {
        const uint32_t x = q / (kGfbLdsSlice / 16u);
        const uint32_t po = t0 + (q % (kGfbLdsSlice / 16u)) * 16u;  // offset inside the packet
        const uint32_t pk = x * a.ps;
        uint32_t v = bv > pk ? bv - pk : 0u;  // valid bytes of this packet
        v = v < a.ps ? v : a.ps;
        stage[r] = load_guarded(base + pk, po, v);
      }
    }
  };
  auto swrite = [&](int b) {
#pragma unroll
    for (int r = 0; r < NQ; ++r) {
      const uint32_t q = tid + (uint32_t)r * kGfbLdsThreads;
      if (q < (uint32_t)kChunks) buf[b][q] = stage[r];
    }
  };
  gload(0);
  swrite(0);
  __syncthreads();
  for (int j = 0; j < a.K; ++j) {
    const int cur = j & 1;
    if (j + 1 < a.K) gload(j + 1);
    LaneVec<LW> y[W];
    const uint32_t* lb = reinterpret_cast<const uint32_t*>(&buf[cur][0]);
#pragma unroll
    for (int x = 0; x < W; ++x) {
      typedef uint32_t v2 __attribute__((ext_vector_type(2)));
      const v2 t = *reinterpret_cast<const v2*>(lb + x * (kGfbLdsSlice / 4u) + tid * 2u);
      y[x].v[0] = t[0];
      y[x].v[1] = t[1];
    }
    uint32_t c[R];
#pragma unroll
    for (int i = 0; i < R; ++i) c[i] = a.coef[i][j];
    gfb_accumulate<W, R, LW, false>(acc, y, c);
    if (j + 1 < a.K) swrite(cur ^ 1);
    __syncthreads();
  }
  if (!active) return;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    uint8_t* p = const_cast<uint8_t*>(a.out[i].base) + o64 * a.out[i].stride;
    const uint32_t bv = a.out[i].valid;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint32_t pk = (uint32_t)x * a.ps;
      lv_store<LW>(p + pk, off, bv > pk ? bv - pk : 0u, acc[i][x]);
    }
  }
}

// ===========================================================================
// Host-side launch templates of these forms.
int gfp_blocks_per_cu();  // resident-grid size of gfp_apply (kernels.hip)

template <int W, int R, bool ACC>
int launch_gfw_t(const GfApply& p, const Chunk& c, hipStream_t s) {
  GfwArgs<R> a;
  uint32_t vmin = 0xFFFFFFFFu;
  a.K = c.nk;
  for (int j = 0; j < kMaxK; ++j) {
    a.in[j] = j < c.nk ? dev_shard(p.in[c.j0 + j], c.o0) : DevShard{nullptr, 0, 0, 0};
    if (j < c.nk) vmin = a.in[j].valid < vmin ? a.in[j].valid : vmin;
  }
  for (int r = 0; r < R; ++r) {
    a.out[r] = dev_shard(p.out[c.r0 + r], c.o0);
    vmin = a.out[r].valid < vmin ? a.out[r].valid : vmin;
    for (int j = 0; j < kMaxK; ++j)
      a.coef[r][j] = j < c.nk ? p.coef[(size_t)(c.r0 + r) * p.K + c.j0 + j] : 0u;
  }
  a.tiles = c.tiles;
  a.vmin = vmin;
  hipLaunchKernelGGL((gfw_apply<W, R, ACC>), dim3((uint32_t)(c.no * c.tiles)), dim3(kThreads), 0,
                     s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

template <int R, bool ACC>
int launch_gf16_t(const GfApply& p, const Chunk& c, hipStream_t s) {
  Gf16Args<R> a;
  uint32_t vmin = 0xFFFFFFFFu;
  a.K = c.nk;
  for (int j = 0; j < kMaxK; ++j) {
    a.in[j] = j < c.nk ? dev_shard(p.in[c.j0 + j], c.o0) : DevShard{nullptr, 0, 0, 0};
    if (j < c.nk) vmin = a.in[j].valid < vmin ? a.in[j].valid : vmin;
  }
  for (int r = 0; r < R; ++r) {
    a.out[r] = dev_shard(p.out[c.r0 + r], c.o0);
    vmin = a.out[r].valid < vmin ? a.out[r].valid : vmin;
    for (int j = 0; j < kMaxK; ++j)
      a.coef[r][j] = j < c.nk ? p.coef[(size_t)(c.r0 + r) * p.K + c.j0 + j] : 0u;
  }
  a.tiles = c.tiles;
  a.vmin = vmin;
  hipLaunchKernelGGL((gf16_apply<R, ACC>), dim3((uint32_t)(c.no * c.tiles)), dim3(kThreads), 0, s,
                     a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

template <int W, int R, bool ACC, int CPT>
int launch_gfp_t(const GfApply& p, const Chunk& c, hipStream_t s) {
  GfpArgs<R> a;
  uint32_t vmin = 0xFFFFFFFFu;
  a.K = c.nk;
  for (int j = 0; j < kMaxK; ++j) {
    a.in[j] = j < c.nk ? dev_shard(p.in[c.j0 + j], c.o0) : DevShard{nullptr, 0, 0, 0};
    if (j < c.nk) vmin = a.in[j].valid < vmin ? a.in[j].valid : vmin;
  }
  for (int r = 0; r < R; ++r) {
    a.out[r] = dev_shard(p.out[c.r0 + r], c.o0);
    vmin = a.out[r].valid < vmin ? a.out[r].valid : vmin;
    for (int j = 0; j < kMaxK; ++j)
      a.coef[r][j] = j < c.nk ? p.coef[(size_t)(c.r0 + r) * p.K + c.j0 + j] : 0u;
  }
  const uint32_t tb = kTileBytes * CPT;
  a.tiles = (uint32_t)((p.block_size + tb - 1) / tb);
  a.vmin = vmin;
  a.total_tiles = (uint32_t)(c.no * a.tiles);
  // resident-sized grid, every block walking the same number of tiles
  const uint32_t cap = (uint32_t)device_cus() * gfp_blocks_per_cu();
  const uint32_t per = (a.total_tiles + cap - 1) / cap;
  const uint32_t grid = (a.total_tiles + per - 1) / per;
  hipLaunchKernelGGL((gfp_apply<W, R, ACC, CPT>), dim3(grid), dim3(kThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

}  // namespace detail
}  // namespace leoec
