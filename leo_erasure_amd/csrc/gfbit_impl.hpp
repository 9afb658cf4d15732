// gfbit_impl.hpp — launch templates of the packet-bitsliced GF(2^w) kernel
// (gfbit_apply, kernels_impl.hpp) shared by gfbit_inst.hip (dispatch and the
// w = 8 measurement forms) and gfbit_w.hip (the shipped launch tables, one
// TU per w so the instances compile in parallel).
#pragma once

#include "kernels_impl.hpp"
#include "knobs.hpp"

namespace leoec {
namespace detail {
// cauchyrs(10,4,8) encode with its bitmatrix compiled in (cbm_inst.hip):
// launches it and returns true when the plan's coefficients are that
// matrix's and Knobs::gfbit_cbm selects it; *rc = the launch's status.
bool launch_cbm(const GfBitApply& p, hipStream_t s, int* rc);
}  // namespace detail

namespace gfbit_detail {

using namespace detail;

using GfbFn = int (*)(const GfBitApply&, int r0, int j0, int nk, uint64_t o0, uint64_t no,
                      hipStream_t);

template <int W, int R, int LW, bool ACC, int PF, bool CEIL = false, int KR = 0,
          int WG = kThreads, int XMAP = 0, int WAVES = 0>
int launch_gfb_t(const GfBitApply& p, int r0, int j0, int nk, uint64_t o0, uint64_t no,
                 hipStream_t s) {
  GfbArgs<R> a;
  a.K = nk;
  a.ps = (uint32_t)(p.block_size / (uint64_t)W);
  a.tiles = packet_tiles(a.ps, WG, 4u * LW);
  for (int j = 0; j < kMaxK; ++j)
    a.in[j] = j < nk ? dev_shard(p.in[j0 + j], o0) : DevShard{nullptr, 0, 0, 0};
  for (int i = 0; i < R; ++i) {
    a.out[i] = dev_shard(p.out[r0 + i], o0);
    for (int j = 0; j < kMaxK; ++j)
      a.coef[i][j] = j < nk ? p.coef[(size_t)(r0 + i) * p.K + j0 + j] : 0u;
  }
  // objects interleaved over the XCDs (xcd_obj_map) for objects of at most
  // kObjMapMaxTiles tiles; Knobs::gfbit_xmap = 0 turns it off (A/B)
  a.xmap = (XMAP == 0 && a.tiles <= kObjMapMaxTiles && knobs().gfbit_xmap != 0) ? 1u : 0u;
  if (KR > 0 && nk > KR) return LEOEC_E_ARG;
  hipLaunchKernelGGL((gfbit_apply<W, R, LW, ACC, PF, CEIL, KR, WG, XMAP, WAVES>),
                     dim3((uint32_t)(no * a.tiles)), dim3(WG), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

constexpr int kPF = 1;  // gfbit_apply: blocks of load look-ahead

template <int W, int LW, int PF = kPF>
GfbFn pick_r(int r, bool acc) {
  static const GfbFn tbl[2][kMaxR] = {
      {&launch_gfb_t<W, 1, LW, false, PF>, &launch_gfb_t<W, 2, LW, false, PF>,
       &launch_gfb_t<W, 3, LW, false, PF>, &launch_gfb_t<W, 4, LW, false, PF>},
      {&launch_gfb_t<W, 1, LW, true, PF>, &launch_gfb_t<W, 2, LW, true, PF>,
       &launch_gfb_t<W, 3, LW, true, PF>, &launch_gfb_t<W, 4, LW, true, PF>}};
  return tbl[acc ? 1 : 0][r - 1];
}

// The shipped launch table of width W (gfbit_w.hip, one TU per W = 2..16).
template <int W>
GfbFn shipped(int r, bool acc);

// gfbk_apply (w = 8, K = 10 inputs, 4 output rows, no accumulation; round 5
// as a measurement form, LEOEC_GFBIT_FORM=5; round 6 shipped for launches
// above kGfbkMinBytes, gfbit_inst.hip): the shipped arithmetic (coefficient bits
// as uniform branches, the bitsliced doubling chain) in the register regime
// of the only access pattern that read 0.77 on this geometry
// (tools/packet_ceiling.hip pattern<4,128>: 16-byte lanes, K compiled in,
// 276 VGPRs = one wave per SIMD with whole blocks of loads in flight).
// Every load is a raw buffer load over the block's resource clipped at its
// valid length (no branch around any load: round 5's liberation finding), a
// ring of LA + 1 blocks keeps LA blocks (8 loads each) in flight, and the
// wave-uniform `full` decision is taken once per tile (edge tiles clear the
// straddling chunk where the packet is consumed).  MASK = 1: coefficient bits
// as v_bitop3 masks instead of branches (twice the XORs, no branch at all).
struct GfbkArgs {
  DevShard in[kMaxK];
  DevShard out[4];
  uint32_t coef[4][kMaxK];
  uint32_t ps;     // packet bytes
  uint32_t vmin;   // smallest valid length over the inputs
  uint32_t tiles;  // tiles per object (over one packet)
  uint32_t xmap;   // 1: xcd_obj_map
};

template <int K, int LA, int WG, bool MASK, bool FULL>
__device__ __forceinline__ void gfbk_tile(const GfbkArgs& a, uint64_t o64, uint32_t off,
                                          bool live) {
  constexpr int W = 8, R = 4, RS = LA + 1;
  auto rs = [&](int j) { return shard_rsrc(a.in[j].base, a.in[j].stride, a.in[j].valid, o64, 16u); };
  u32x4 ring[RS][W];
  auto load = [&](int j, u32x4 (&y)[W]) {
    const auto r = rs(j);
#pragma unroll
    for (int x = 0; x < W; ++x) y[x] = libb_load(r, off + (uint32_t)x * a.ps);
  };
  u32x4 acc[R][W];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int x = 0; x < W; ++x) acc[i][x] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int u = 0; u < LA && u < K; ++u) load(u, ring[u]);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (j + LA < K) load(j + LA, ring[(j + LA) % RS]);
    u32x4(&y)[W] = ring[j % RS];
    if (!FULL) {
#pragma unroll
      for (int x = 0; x < W; ++x) y[x] = libb_clip(y[x], a.in[j].valid, off + (uint32_t)x * a.ps);
    }
    uint32_t c[R];
#pragma unroll
    for (int i = 0; i < R; ++i) c[i] = a.coef[i][j];
#pragma unroll
    for (int t = 0; t < W; ++t) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        if (MASK) {
          const uint32_t m = 0u - ((c[i] >> t) & 1u);
#pragma unroll
          for (int x = 0; x < W; ++x)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc[i][x][e] = __builtin_amdgcn_bitop3_b32(acc[i][x][e], y[x][e], m, 0x6A);
        } else if ((c[i] >> t) & 1u) {
#pragma unroll
          for (int x = 0; x < W; ++x) acc[i][x] ^= y[x];
        }
      }
      if (t + 1 < W) {  // y <- y * 2 (poly 0x11D: taps at bits 2, 3, 4)
        const u32x4 top = y[W - 1];
#pragma unroll
        for (int r = W - 1; r >= 1; --r)
          y[r] = ((DefaultPoly<W>::v >> r) & 1u) ? (y[r - 1] ^ top) : y[r - 1];
        y[0] = top;
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // the next block's loads stay where the ring puts them
  }
  if (!live) return;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    uint8_t* b = const_cast<uint8_t*>(a.out[i].base) + o64 * a.out[i].stride;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint32_t at = off + (uint32_t)x * a.ps;
      if (FULL) st16<true>(b + at, acc[i][x]);
      else store_guarded(b + (uint32_t)x * a.ps, off, packet_valid(a.out[i].valid, x, a.ps), acc[i][x]);
    }
  }
}

template <int K, int LA, int WG, bool MASK, int WAVES>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(WAVES, 8)))
gfbk_apply(const GfbkArgs a) {
  constexpr uint32_t TB = WG * 16u;
  const uint32_t bid = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t t0 = tile * TB;
  const uint32_t off = t0 + threadIdx.x * 16u;
  // wave-uniform: the tile lies inside every packet of every input
  const bool full = t0 + TB <= a.ps && 7ull * a.ps + t0 + TB <= (uint64_t)a.vmin;
  if (full) gfbk_tile<K, LA, WG, MASK, true>(a, obj, off, true);
  else gfbk_tile<K, LA, WG, MASK, false>(a, obj, off, off < a.ps);
}

template <int LA, int WG, bool MASK, int WAVES>
int launch_gfbk_t(const GfBitApply& p, int r0, int j0, int nk, uint64_t o0, uint64_t no,
                  hipStream_t s) {
  GfbkArgs a;
  a.ps = (uint32_t)(p.block_size / 8u);
  a.tiles = packet_tiles(a.ps, WG, 16u);
  a.vmin = 0xFFFFFFFFu;
  for (int j = 0; j < kMaxK; ++j) {
    a.in[j] = j < nk ? dev_shard(p.in[j0 + j], o0) : DevShard{nullptr, 0, 0, 0};
    if (j < nk && a.in[j].valid < a.vmin) a.vmin = a.in[j].valid;
  }
  for (int i = 0; i < 4; ++i) {
    a.out[i] = dev_shard(p.out[r0 + i], o0);
    for (int j = 0; j < kMaxK; ++j)
      a.coef[i][j] = j < nk ? p.coef[(size_t)(r0 + i) * p.K + j0 + j] : 0u;
  }
  a.xmap = (a.tiles <= kObjMapMaxTiles && knobs().gfbit_xmap != 0) ? 1u : 0u;
  hipLaunchKernelGGL((gfbk_apply<10, LA, WG, MASK, WAVES>), dim3((uint32_t)(no * a.tiles)),
                     dim3(WG), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

// The shipped gfbk form: 64 lanes, 3 blocks of loads in flight, one wave per
// SIMD allowed.  It reads 0.742-0.747 of 8 TB/s on cauchyrs(10,4,8) encode at
// 3,072-8,192 x 1 MiB objects against 0.707-0.714 for gfbit_apply (+4.6 to
// +5.1 %), decode +2.2 to +2.6 %, repair within -0.9 to +2.4 %; at 2,048
// objects +1.6 / +1.0 / -1.5 %, at 1,024 -2.6 to -3.8 % (one wave per SIMD
// leaves a small launch's tail exposed): profiles/r06_s1_ab_cauchy_*.log,
// r06_s2_ab_cauchy_*.log, interleaved in one process.  So launches of at
// least kGfbkMinBytes algorithmic bytes take it.
constexpr uint64_t kGfbkMinBytes = 4000000000ull;  // between 2,048 (3.0 GB) and 3,072 (4.5 GB) objects
inline bool gfbk_pays(const GfBitApply& p, int r, bool acc, int nk, uint64_t no) {
  const uint64_t min_bytes =
#ifdef LEOEC_MEASURE
      knobs().gfbk_min_mib >= 0 ? (uint64_t)knobs().gfbk_min_mib << 20 :
#endif
                                kGfbkMinBytes;
  return p.w == 8 && r == 4 && !acc && nk == 10 &&
         no * (uint64_t)(nk + r) * p.block_size >= min_bytes;
}

#ifdef LEOEC_MEASURE
template <int R>
struct Gfb2Args {
  InCol col[kMaxK + 1];  // col[K]: empty (valid 0), the target of the last prefetch
  DevShard out[R];
  int K;
  uint32_t ps;     // packet bytes
  uint32_t bs;     // block bytes (w packets)
  uint32_t tiles;  // tiles per object (over one packet)
  uint32_t xmap;   // 1: xcd_obj_map
};

// Packet x of the block behind rs: this lane's 4*LW bytes at off.
template <int W, int LW>
__device__ __forceinline__ void gfb2_load(__amdgpu_buffer_rsrc_t rs, uint32_t ps, uint32_t off,
                                          LaneVec<LW> (&y)[W]) {
#pragma unroll
  for (int x = 0; x < W; ++x) {
    const uint32_t vo = off + (uint32_t)x * ps;
    if constexpr (LW == 4) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 2);
#pragma unroll
      for (int e = 0; e < 4; ++e) y[x].v[e] = v[e];
    } else if constexpr (LW == 2) {
      typedef uint32_t v2 __attribute__((ext_vector_type(2)));
      const v2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, vo, 0, 2);
      y[x].v[0] = v[0];
      y[x].v[LW - 1] = v[1];
    } else {
      y[x].v[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 2);
    }
  }
}

// Bytes at or past the block's valid length cleared (blocks shorter than bs).
template <int W, int LW>
__device__ __forceinline__ void gfb2_tail(uint32_t valid, uint32_t ps, uint32_t off,
                                          LaneVec<LW> (&y)[W]) {
#pragma unroll
  for (int x = 0; x < W; ++x) {
    const uint32_t p = off + (uint32_t)x * ps;
    const uint32_t n = p >= valid ? 0u : (valid - p > 4u * LW ? 4u * LW : valid - p);
#pragma unroll
    for (int e = 0; e < LW; ++e) {
      const uint32_t lo = 4u * e;
      y[x].v[e] &= n >= lo + 4u ? 0xFFFFFFFFu : (n <= lo ? 0u : (1u << (8u * (n - lo))) - 1u);
    }
  }
}

// (takes no reference to the kernel argument block: one would make the
// compiler read the arguments through vector loads, and the buffer resources
// built from them divergent)
template <int W, int R, int LW>
__device__ __forceinline__ void gfb2_step(uint32_t bs, uint32_t ps, const InCol& col, uint32_t off,
                                          LaneVec<LW> (&y)[W], LaneVec<LW> (&acc)[R][W]) {
  if (col.valid < bs) gfb2_tail<W, LW>(col.valid, ps, off, y);
  uint32_t c[R];
#pragma unroll
  for (int i = 0; i < R; ++i) c[i] = col.coef[i];
  gfb_accumulate<W, R, LW, false>(acc, y, c);
}

template <int W, int R, int LW, bool ACC, int PF, int WG = kThreads>
__global__ void __launch_bounds__(WG) gfb2_apply(const Gfb2Args<R> a) {
  constexpr uint32_t LB = 4u * LW;
  const uint32_t bid = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t off = tile * (WG * LB) + threadIdx.x * LB;
  // lanes past the packet (last tile) compute on whatever they read and do
  // not store: an early return here made the compiler treat the loop's
  // buffer resources as divergent
  const bool live = off < a.ps;
  const uint64_t o64 = obj;
  LaneVec<LW> acc[R][W];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int x = 0; x < W; ++x) {
      if (ACC && live) {
        const uint32_t pk = (uint32_t)x * a.ps;
        const uint32_t bv = a.out[i].valid;
        acc[i][x] = lv_load<LW>(a.out[i].base + o64 * a.out[i].stride + pk, off,
                                bv > pk ? bv - pk : 0u);
      } else {
#pragma unroll
        for (int e = 0; e < LW; ++e) acc[i][x].v[e] = 0u;
      }
    }
  const int K = a.K;
  if constexpr (PF == 0) {
    // load, then compute: no second buffer (the prefetching loop below
    // needs ~64 more VGPRs, i.e. 2 waves per SIMD instead of 4)
    LaneVec<LW> y[W];
    InCol cur = a.col[0];
    for (int j = 0; j < K; ++j) {
      gfb2_load<W, LW>(shard_rsrc(cur.base, cur.stride, cur.valid, o64, LB), a.ps, off, y);
      const InCol nx = a.col[j + 1];  // col[K] is the empty record
      gfb2_step<W, R, LW>(a.bs, a.ps, cur, off, y, acc);
      cur = nx;
    }
  } else {
    LaneVec<LW> ya[W], yb[W];
    InCol cur = a.col[0], nx = a.col[K > 1 ? 1 : K];
    gfb2_load<W, LW>(shard_rsrc(cur.base, cur.stride, cur.valid, o64, LB), a.ps, off, ya);
    for (int j = 0;; j += 2) {
      gfb2_load<W, LW>(shard_rsrc(nx.base, nx.stride, nx.valid, o64, LB), a.ps, off, yb);
      const InCol nx2 = a.col[j + 2 < K ? j + 2 : K];
      gfb2_step<W, R, LW>(a.bs, a.ps, cur, off, ya, acc);
      __builtin_amdgcn_sched_barrier(0);  // keep the next loads below: same registers
      if (j + 1 >= K) break;
      gfb2_load<W, LW>(shard_rsrc(nx2.base, nx2.stride, nx2.valid, o64, LB), a.ps, off, ya);
      const InCol nx3 = a.col[j + 3 < K ? j + 3 : K];
      gfb2_step<W, R, LW>(a.bs, a.ps, nx, off, yb, acc);
      __builtin_amdgcn_sched_barrier(0);
      if (j + 2 >= K) break;
      cur = nx2;
      nx = nx3;
    }
  }
  if (!live) return;
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

template <int W, int R, int LW, bool ACC, int PF, int WG = kThreads>
int launch_gfb2_t(const GfBitApply& p, int r0, int j0, int nk, uint64_t o0, uint64_t no,
                  hipStream_t s) {
  static_assert(LW == 1 || LW == 2 || LW == 4, "gfb2_apply lane width");
  Gfb2Args<R> a;
  a.K = nk;
  a.bs = (uint32_t)p.block_size;
  a.ps = (uint32_t)(p.block_size / (uint64_t)W);
  constexpr uint32_t tb = WG * 4u * LW;
  a.tiles = (a.ps + tb - 1) / tb;
  for (int x = 0; x <= kMaxK; ++x) {
    InCol& col = a.col[x];
    col = InCol{};
    if (x < nk) {
      const DevShard d = dev_shard(p.in[j0 + x], o0);
      col.base = d.base;
      col.stride = d.stride;
      col.valid = d.valid;
      for (int i = 0; i < R; ++i) col.coef[i] = p.coef[(size_t)(r0 + i) * p.K + j0 + x];
    } else {
      col.base = a.col[0].base;  // empty range: never dereferenced
    }
  }
  for (int i = 0; i < R; ++i) a.out[i] = dev_shard(p.out[r0 + i], o0);
  a.xmap = (a.tiles <= kObjMapMaxTiles && knobs().gfbit_xmap != 0) ? 1u : 0u;
  hipLaunchKernelGGL((gfb2_apply<W, R, LW, ACC, PF, WG>), dim3((uint32_t)(no * a.tiles)),
                     dim3(WG), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

constexpr int kPF2 = 0;  // gfb2_apply: load-then-compute (LEOEC_GFBIT_PF=1: prefetching loop)

template <int W, int LW, int PF = kPF2, int WG = kThreads>
GfbFn pick_r2(int r, bool acc) {
  static const GfbFn tbl[2][kMaxR] = {
      {&launch_gfb2_t<W, 1, LW, false, PF, WG>, &launch_gfb2_t<W, 2, LW, false, PF, WG>,
       &launch_gfb2_t<W, 3, LW, false, PF, WG>, &launch_gfb2_t<W, 4, LW, false, PF, WG>},
      {&launch_gfb2_t<W, 1, LW, true, PF, WG>, &launch_gfb2_t<W, 2, LW, true, PF, WG>,
       &launch_gfb2_t<W, 3, LW, true, PF, WG>, &launch_gfb2_t<W, 4, LW, true, PF, WG>}};
  return tbl[acc ? 1 : 0][r - 1];
}

// gfb2_apply's launch table of width W (gfbit_w.hip).
template <int W>
GfbFn measure2(int r, bool acc);

// The measurement form the LEOEC_GFBIT_* knobs select for this launch
// (gfbit_measure.hip), or nullptr for the shipped form.
GfbFn pick_measure(const GfBitApply& p, int w, int r, bool acc, int nk, bool big);
#endif  // LEOEC_MEASURE

}  // namespace gfbit_detail
}  // namespace leoec
