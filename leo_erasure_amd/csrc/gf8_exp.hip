// gf8_exp.hip — measurement variants of gf8_apply<10, 4> (the RS(10,4,8)
// headline shape), selected with LEOEC_GF8_VARIANT=<n> for A/B runs in one
// process (tools/kvariants.py).  Variant 1 is the shipped configuration.
#include "kernels_impl.hpp"

namespace leoec {
namespace detail {

// Compiled once per part (-DLEOEC_GF8_EXP_PART=0..3, variant n in part n % 4)
// so the measurement build's variants compile in parallel.
#ifndef LEOEC_GF8_EXP_PART
#error "compile with -DLEOEC_GF8_EXP_PART=<0..3>"
#endif

#if LEOEC_GF8_EXP_PART == 3
// Variant 47 (measurement only): pair-swapped block halves.  A 128-lane
// workgroup covers two 1 KiB windows of every block; wave w loads inputs
// 0..K/2-1 at its own window and inputs K/2..K-1 at the partner's window,
// so no wave's burst holds block j and block j+K/2 of one column (at the
// 64 MiB geometry those sit 32 MiB + 128 B apart, on the same HBM channels:
// DESIGN.md, "Why 64 MiB objects read less").  Each wave multiplies what it
// loaded, hands the partner's half-sums over through LDS, and stores its
// own window.  K = 10, R = 4, no accumulation.
template <int K, int R>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(3, 8)))
gf8_swap_apply(const Gf8Args<K, R> a) {
  __shared__ Gf8Lds<K, R> lds;
  __shared__ u32x4 part[2][R][64];
  for (uint32_t i = threadIdx.x; i < (uint32_t)(R * K); i += blockDim.x) {
    const uint32_t* t = a.tab[i / K][i % K];
    lds.t[i][0] = u32x4{t[0], t[1], t[2], t[3]};
    lds.t[i][1] = u32x4{t[4], 0u, 0u, 0u};
  }
  __syncthreads();
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64u);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t obj = blockIdx.x / a.tiles;
  const uint32_t base = (blockIdx.x - obj * a.tiles) * 2048u;
  const uint32_t myoff = base + wv * 1024u + lane * 16u;
  const uint32_t ptoff = base + (1u - wv) * 1024u + lane * 16u;
  const bool full = base + 2048u <= a.vmin;  // wave-uniform
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t off = j < K / 2 ? myoff : ptoff;
    const uint8_t* p = a.in[j].base + (uint64_t)obj * a.in[j].stride;
    d[j] = full ? ld16<true>(p + off) : load_guarded(p, off, a.in[j].valid);
  }
  u32x4 acc[R], oth[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = oth[r] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < K; ++j) {
    uint32_t s0[4], s1[4], s2[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t x = d[j][e];
      s0[e] = x & 0x07070707u;
      s1[e] = (x >> 3) & 0x07070707u;
      s2[e] = (x >> 6) & 0x03030303u;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32x4 t = lds.t[r * K + j][0];
      const uint32_t t2 = lds.t[r * K + j][1][0];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t v = xor3(perm(t[1], t[0], s0[e]), perm(t[3], t[2], s1[e]), perm(t2, t2, s2[e]));
        if (j < K / 2) acc[r][e] ^= v;
        else oth[r][e] ^= v;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) part[wv][r][lane] = oth[r];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    acc[r] ^= part[1u - wv][r][lane];
    uint8_t* q = const_cast<uint8_t*>(a.out[r].base) + (uint64_t)obj * a.out[r].stride;
    if (full) st16<true>(q + myoff, acc[r]);
    else store_guarded(q, myoff, a.out[r].valid, acc[r]);
  }
}

int launch_gf8_swap(const GfApply& p, const Chunk& c, hipStream_t s) {
  constexpr int K = 10, R = 4;
  if (c.nk != K || c.nr != R || c.j0 != 0) return LEOEC_E_ARG;
  Gf8Args<K, R> a;
  a.one = a.zero = 0;
  uint32_t vmin = 0xFFFFFFFFu;
  for (int j = 0; j < K; ++j) {
    a.in[j] = dev_shard(p.in[c.j0 + j], c.o0);
    vmin = a.in[j].valid < vmin ? a.in[j].valid : vmin;
  }
  for (int r = 0; r < R; ++r) {
    a.out[r] = dev_shard(p.out[c.r0 + r], c.o0);
    vmin = a.out[r].valid < vmin ? a.out[r].valid : vmin;
    for (int j = 0; j < K; ++j)
      gf8_tables(p.coef[(size_t)(c.r0 + r) * p.K + c.j0 + j] & 0xFFu, a.tab[r][j]);
  }
  a.tiles = (uint32_t)((p.block_size + 2047u) / 2048u);
  a.vmin = vmin;
  a.total_tiles = (uint32_t)(c.no * a.tiles);
  a.nobj = (uint32_t)c.no;
  a.tmap = 0;
  a.tperm = 1;
  hipLaunchKernelGGL((gf8_swap_apply<K, R>), dim3(a.total_tiles), dim3(128), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}
#endif

template <>
ChunkFn gf8_variant_part<LEOEC_GF8_EXP_PART>(int v) {
  //                             K   R  ACC    CPT NT    BR  COPY   PIPE   LDS
  switch (v) {
#if LEOEC_GF8_EXP_PART == 0
    case 4: return &launch_gf8_t<10, 4, false, 1, true, 1, false, false, true>;   // branchy lds
    case 12: return &launch_gf8_t<10, 4, false, 1, false, 0, false, false, true>; // no nt
    case 16: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 6>;  // >=6 waves
    case 20: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 512>;
    case 24: return &launch_gf8_t<10, 4, false, 1, true, 1, true, false, false, 5, 256, 1>;  // copy xmap
    case 28: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 4, 64>;   // wg64 >=4 waves
    case 32: return &launch_gf8_t<10, 4, false, 1, true, -1, false, false, true, 5, 256, 2, true>; // buffer, auto branchy
    case 36: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 0, false, false, true>;  // loads before LDS staging
#endif
#if LEOEC_GF8_EXP_PART == 1
    case 1: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true>;   // shipped
    case 5: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, false>;  // paired sgpr
    case 17: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 8>;  // 8 waves
    case 21: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 1>;
    case 25: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 64>;   // wg64
    case 33: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 2, false, true>;  // row 0 / column 0 of ones folded
    case 37: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 0, true, false, true>;   // + buffer ld/st
    case 29: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 6, 64>;   // wg64 >=6 waves
#endif
#if LEOEC_GF8_EXP_PART == 2
    case 2: return &launch_gf8_t<10, 4, false, 2, true, 0, false, false, true>;   // cpt2
    case 22: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 512, 1>;
    case 26: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 128>;  // wg128
    case 30: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 2, true>;  // buffer ld/st
    case 34: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 2>;  // xcd_obj_map always
#endif
#if LEOEC_GF8_EXP_PART == 3
    case 3: return &launch_gf8_t<10, 4, false, 1, true, 1, false, false, false>;  // branchy sgpr
    case 7: return &launch_gf8_t<10, 4, false, 1, true, 1, true, false, false>;   // copy-xor
    case 15: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5>;  // >=5 waves
    case 23: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 1024>;
    case 27: return &launch_gf8_t<10, 4, false, 1, true, 1, true, false, false, 5, 64>;   // copy wg64
    case 31: return &launch_gf8_t<10, 4, false, 1, true, 1, true, false, false, 5, 256, 2, true>;  // copy buffer
    case 35: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 64, 0, true>;  // buffer ld/st wg64, run-time tile map
    case 47: return &launch_gf8_swap;  // pair-swapped block halves, LDS hand-over
    case 39: return &launch_gf8_t<10, 4, false, 1, true, 0, true, false, true>;   // copy, shipped shape
    case 43: return &launch_gf8_t<10, 4, false, 1, true, 0, true, false, true, 5, 64>;   // copy, shipped shape, wg64
#endif
    default: return nullptr;
  }
}

#if LEOEC_GF8_EXP_PART == 0
ChunkFn gf8_variant(int v) {
  if (v <= 0) return nullptr;
  switch (v % 4) {
    case 0: return gf8_variant_part<0>(v);
    case 1: return gf8_variant_part<1>(v);
    case 2: return gf8_variant_part<2>(v);
    default: return gf8_variant_part<3>(v);
  }
}
#endif

}  // namespace detail
}  // namespace leoec
