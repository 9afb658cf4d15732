// gfbit_measure.hip — measurement library only (-DLEOEC_MEASURE): the A/B
// forms of the packet-bitsliced GF(2^w) kernel (cauchyrs), selected with the
// LEOEC_GFBIT_* knobs through pick_measure(); the shipped form and its
// dispatch are gfbit_inst.hip / gfbit_w.hip.  None of these ship (DESIGN.md
// §Measured, cauchyrs, has what each read).
//
// gfb2_apply (LEOEC_GFBIT_FORM=1, gfbit_impl.hpp) is the shipped arithmetic
// with the gfs_apply loading scheme: unconditional raw-buffer loads
// (shard_rsrc) and per-input 64-byte argument records fetched one input
// ahead.  gfbit_apply's guarded loads are per-lane branches after which the
// compiler waits for every outstanding load, so its look-ahead overlaps
// nothing; it hides latency with occupancy instead (132 VGPRs).  The
// buffer-load form measured lower on cauchyrs(10,4,8) 1 MiB
// (profiles/r02_v11_ab_gfb2.log: 0.684 / 0.682 load-then-compute at 120
// VGPRs, 0.699 / 0.686 with the next block in flight at 184 VGPRs, against
// 0.711 / 0.703).
#ifndef LEOEC_MEASURE
#error "gfbit_measure.hip belongs to the measurement library (-DLEOEC_MEASURE)"
#endif

#include "gfbit_impl.hpp"

namespace leoec {

using namespace detail;

namespace gfbit_detail {

namespace {
// gfbx_apply (measurement form, LEOEC_GFBIT_FORM=2; w = 8, 4 output rows,
// <= 16 inputs): 16-byte lanes without the 16-byte lanes' register bill.  A
// 128-lane workgroup covers 1 KiB of x in every packet; both waves work on
// the same 64 columns.  Per input block, wave v loads packets 4v..4v+3
// (1 KiB contiguous each, raw buffer loads: out-of-range reads return 0) and
// writes them to LDS; after one barrier each wave reads all 8 packets of its
// columns back and accumulates output rows 2v, 2v+1 only (acc 2 x 8 x 4 =
// 64 VGPRs instead of 128).  LDS is double-buffered so the barrier of block
// j also retires every read of block j-1's buffer, and block j+1's loads are
// in flight while block j is computed.
constexpr int kGfbxLanes = 64;                     // columns per workgroup
constexpr uint32_t kGfbxSlice = kGfbxLanes * 16u;  // bytes of x per tile

template <int W>
__global__ void __launch_bounds__(2 * kGfbxLanes) gfbx_apply(const GfbArgs<4> a) {
  static_assert(W % 2 == 0, "two waves split the packets");
  constexpr int HP = W / 2;  // packets loaded per wave
  __shared__ u32x4 lds[2][W][kGfbxLanes];
  const uint32_t lane = threadIdx.x % kGfbxLanes;
  const uint32_t v = __builtin_amdgcn_readfirstlane(threadIdx.x / kGfbxLanes);
  const uint32_t bid = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t off = tile * kGfbxSlice + lane * 16u;
  const bool live = off < a.ps;
  const uint64_t o64 = obj;
  const int K = a.K;
  u32x4 p[HP];
  auto load = [&](int j) {
    const DevShard d = a.in[j];
    const auto rs = shard_rsrc(d.base, d.stride, d.valid, o64, 16u);
#pragma unroll
    for (int h = 0; h < HP; ++h) {
      const uint32_t x = v * HP + h;
      const uint32_t at = x * a.ps + off;
      u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(rs, at, 0, 2);
      if (d.valid < at + 16u) t = keep_first(t, d.valid > at ? d.valid - at : 0u);
      p[h] = t;
    }
  };
  LaneVec<4> acc[2][W];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int x = 0; x < W; ++x)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[i][x].v[e] = 0u;
  load(0);
  for (int j = 0; j < K; ++j) {
    const int b = j & 1;
#pragma unroll
    for (int h = 0; h < HP; ++h) lds[b][v * HP + h][lane] = p[h];
    __syncthreads();
    if (j + 1 < K) load(j + 1);
    LaneVec<4> y[W];
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const u32x4 t = lds[b][x][lane];
#pragma unroll
      for (int e = 0; e < 4; ++e) y[x].v[e] = t[e];
    }
    uint32_t c[2];
    c[0] = a.coef[2 * v][j];
    c[1] = a.coef[2 * v + 1][j];
    gfb_accumulate<W, 2, 4, false>(acc, y, c);
  }
  if (!live) return;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const DevShard d = a.out[2 * v + i];
    uint8_t* q = const_cast<uint8_t*>(d.base) + o64 * d.stride;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint32_t pk = (uint32_t)x * a.ps;
      lv_store<4>(q + pk, off, d.valid > pk ? d.valid - pk : 0u, acc[i][x]);
    }
  }
}

int launch_gfbx_8(const GfBitApply& p, int r0, int j0, int nk, uint64_t o0, uint64_t no,
                  hipStream_t s) {
  GfbArgs<4> a;
  a.K = nk;
  a.ps = (uint32_t)(p.block_size / 8u);
  a.tiles = (a.ps + kGfbxSlice - 1) / kGfbxSlice;
  for (int j = 0; j < kMaxK; ++j)
    a.in[j] = j < nk ? dev_shard(p.in[j0 + j], o0) : DevShard{nullptr, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    a.out[i] = dev_shard(p.out[r0 + i], o0);
    for (int j = 0; j < kMaxK; ++j)
      a.coef[i][j] = j < nk ? p.coef[(size_t)(r0 + i) * p.K + j0 + j] : 0u;
  }
  a.xmap = (a.tiles <= kObjMapMaxTiles && knobs().gfbit_xmap != 0) ? 1u : 0u;
  hipLaunchKernelGGL((gfbx_apply<8>), dim3((uint32_t)(no * a.tiles)), dim3(2 * kGfbxLanes), 0, s,
                     a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

// gfba_apply (measurement form, LEOEC_GFBIT_FORM=3; no accumulation, <= 16
// inputs, every input's valid length a multiple of 16): the shipped
// arithmetic (8-byte lanes, 64 accumulator VGPRs) fed by line-aligned
// loads.  At the reference's 1 MiB geometry ps = 13,120 B, so odd packets
// start mid cache line and every 512-B wave load of one touches 5 lines
// instead of 4 (tools/packet_ceiling.hip: the same access pattern on
// 128-B-aligned packets reads 0.756 against 0.69-0.72).  Each wave owns a
// 512-B column of every packet; per input block it copies, for each packet,
// the 128-B lines covering its column (5 lines when the column starts mid
// line, 4 otherwise) into its own LDS slot with 16-byte buffer-to-LDS loads
// (no VGPRs held by the copy), then reads its 8 bytes per lane from the slot
// at the column's phase.  Two slots per packet: block j+1's copy is in
// flight while block j is computed.  Waves never share LDS: no barriers.
constexpr uint32_t kGfbaCol = 512;           // bytes of a packet per wave (64 lanes x 8 B)
constexpr uint32_t kGfbaSlot = kGfbaCol + 128;  // lines covering a column at any 16-B phase

template <int W, int R, int WG, bool CEIL, int NB>
__global__ void __launch_bounds__(WG) gfba_apply(const GfbArgs<R> a) {
  static_assert(NB >= 2 && NB <= 6, "slots per packet");
  __shared__ __attribute__((aligned(16))) uint8_t lds[WG / 64][NB][W][kGfbaSlot];
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64u);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t bid = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t col0 = tile * (WG / 64u) * kGfbaCol + wv * kGfbaCol;
  if (col0 >= a.ps) return;  // wave-uniform: no barriers below
  const uint64_t o64 = obj;
  const int K = a.K;
  // start of the lines holding packet x's column, and the column's phase in them
  auto phase = [&](const DevShard& d, int x) -> uint32_t {
    const uint64_t at = (uint64_t)(uintptr_t)(d.base + o64 * d.stride) + (uint64_t)x * a.ps + col0;
    return __builtin_amdgcn_readfirstlane((uint32_t)at & 127u);
  };
  // W copies per block (one per packet, lanes past the lines masked off)
  auto issue = [&](int j, int b) {
    const DevShard d = a.in[j];
    const auto rs = shard_rsrc(d.base, d.stride, d.valid, o64, 16u);
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint32_t sh = phase(d, x);
      const uint32_t nl = sh ? (kGfbaCol + 128u) / 16u : kGfbaCol / 16u;
      // an offset below the shard's start wraps past its range and reads zeros
      const uint32_t vo = (uint32_t)x * a.ps + col0 - sh + lane * 16u;
      if (lane < nl)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)&lds[wv][b][x][0], 16, vo, 0, 0, 2);
    }
  };
  LaneVec<2> acc[R][W];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int x = 0; x < W; ++x) acc[i][x].v[0] = acc[i][x].v[1] = 0u;
#pragma unroll
  for (int u = 0; u < NB - 1; ++u)
    if (u < K) issue(u, u);
  int b = 0;
  for (int j = 0; j < K; ++j) {
    // block j's copies landed; the next min(NB-2, K-1-j) blocks' stay in flight
    const int ahead = K - 1 - j < NB - 2 ? K - 1 - j : NB - 2;
    if (NB == 2 || ahead == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W) : "memory");
    else if (NB == 3 || ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * W) : "memory");
    else if (NB == 4 || ahead == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * W) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * W) : "memory");
    // the reads are inline asm: for a plain LDS read the compiler waits for
    // every copy in flight (vmcnt(0)), draining the ring; their results are
    // tied to the lgkmcnt wait below so nothing uses them earlier
    static_assert(W == 8, "gfba_apply: eight packets per block");
    uint64_t t[W];
    const DevShard d = a.in[j];
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint32_t sh = phase(d, x);
      const auto lp = (__attribute__((address_space(3))) const uint8_t*)&lds[wv][b][x][sh + lane * 8u];
      asm volatile("ds_read_b64 %0, %1" : "=v"(t[x]) : "v"((uint32_t)(size_t)lp));
    }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]),
                   "+v"(t[6]), "+v"(t[7]));
    LaneVec<2> y[W];
#pragma unroll
    for (int x = 0; x < W; ++x) {
      y[x].v[0] = (uint32_t)t[x];
      y[x].v[1] = (uint32_t)(t[x] >> 32);
    }
    // the slot block j-1 used is free (its reads were consumed last iteration)
    if (j + NB - 1 < K) issue(j + NB - 1, b == 0 ? NB - 1 : b - 1);
    b = b + 1 == NB ? 0 : b + 1;
    uint32_t c[R];
#pragma unroll
    for (int i = 0; i < R; ++i) c[i] = a.coef[i][j];
    gfb_accumulate<W, R, 2, CEIL>(acc, y, c);
  }
  const uint32_t off = col0 + lane * 8u;
  if (off >= a.ps) return;  // (ps is a multiple of 16: off < ps => all 8 bytes in the packet)
#pragma unroll
  for (int i = 0; i < R; ++i) {
    uint8_t* p = const_cast<uint8_t*>(a.out[i].base) + o64 * a.out[i].stride;
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint32_t pk = (uint32_t)x * a.ps;
      lv_store<2>(p + pk, off, packet_valid(a.out[i].valid, x, a.ps), acc[i][x]);
    }
  }
}

// gfba_apply applies: w = 8, no accumulation, every input's valid length a
// multiple of 16 (the copy's range check then zero-fills exactly the bytes
// past it).
bool gfba_applies(const GfBitApply& p, int w, bool acc, int nk) {
  if (w != 8 || acc || nk > kMaxK) return false;
  for (const Shard& sh : p.in)
    if (sh.valid % 16u) return false;
  return true;
}

template <int R, int WG, bool CEIL, int NB>
int launch_gfba_t(const GfBitApply& p, int r0, int j0, int nk, uint64_t o0, uint64_t no,
                  hipStream_t s) {
  GfbArgs<R> a;
  a.K = nk;
  a.ps = (uint32_t)(p.block_size / 8u);
  a.tiles = (a.ps + (WG / 64u) * kGfbaCol - 1u) / ((WG / 64u) * kGfbaCol);
  for (int j = 0; j < kMaxK; ++j)
    a.in[j] = j < nk ? dev_shard(p.in[j0 + j], o0) : DevShard{nullptr, 0, 0, 0};
  for (int i = 0; i < R; ++i) {
    a.out[i] = dev_shard(p.out[r0 + i], o0);
    for (int j = 0; j < kMaxK; ++j)
      a.coef[i][j] = j < nk ? p.coef[(size_t)(r0 + i) * p.K + j0 + j] : 0u;
  }
  a.xmap = (a.tiles <= kObjMapMaxTiles && knobs().gfbit_xmap != 0) ? 1u : 0u;
  hipLaunchKernelGGL((gfba_apply<8, R, WG, CEIL, NB>), dim3((uint32_t)(no * a.tiles)), dim3(WG),
                     0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

template <int WG, bool CEIL, int NB>
GfbFn pick_gfba(int r) {
  static const GfbFn tbl[kMaxR] = {&launch_gfba_t<1, WG, CEIL, NB>, &launch_gfba_t<2, WG, CEIL, NB>,
                                   &launch_gfba_t<3, WG, CEIL, NB>, &launch_gfba_t<4, WG, CEIL, NB>};
  return tbl[r - 1];
}

GfbFn pick_gfba_knobs(int r) {
  const Knobs& kn = knobs();
  // LEOEC_GFBIT_PF = blocks in flight (1..3: 2..4 slots per packet);
  // LEOEC_GFBIT_WG=256: four waves per workgroup (each its own slots);
  // LEOEC_GFBIT_CEIL=1: XOR-only memory form (not a code)
  const int pf = kn.gfbit_pf;
  if (kn.gfbit_wg == 256) {
    if (kn.gfbit_ceil) return pick_gfba<256, true, 2>(r);
    return pick_gfba<256, false, 2>(r);
  }
  if (kn.gfbit_ceil) return pf >= 3 ? pick_gfba<64, true, 4>(r) : pf == 2 ? pick_gfba<64, true, 3>(r) : pick_gfba<64, true, 2>(r);
  if (pf >= 5) return pick_gfba<64, false, 6>(r);
  if (pf == 4) return pick_gfba<64, false, 5>(r);
  if (pf == 3) return pick_gfba<64, false, 4>(r);
  if (pf == 2) return pick_gfba<64, false, 3>(r);
  return pick_gfba<64, false, 2>(r);
}

template <int W, int R, bool ACC>
int launch_gfb_lds_t(const GfBitApply& p, int r0, int j0, int nk, uint64_t o0, uint64_t no,
                     hipStream_t s) {
  GfbArgs<R> a;
  a.K = nk;
  a.ps = (uint32_t)(p.block_size / (uint64_t)W);
  a.tiles = (a.ps + kGfbLdsSlice - 1) / kGfbLdsSlice;
  a.xmap = 0;
  for (int j = 0; j < kMaxK; ++j)
    a.in[j] = j < nk ? dev_shard(p.in[j0 + j], o0) : DevShard{nullptr, 0, 0, 0};
  for (int i = 0; i < R; ++i) {
    a.out[i] = dev_shard(p.out[r0 + i], o0);
    for (int j = 0; j < kMaxK; ++j)
      a.coef[i][j] = j < nk ? p.coef[(size_t)(r0 + i) * p.K + j0 + j] : 0u;
  }
  hipLaunchKernelGGL((gfbit_lds_apply<W, R, ACC>), dim3((uint32_t)(no * a.tiles)),
                     dim3(kGfbLdsThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

// Measurement forms of the w = 8 kernel (Knobs::gfbit_*): lane width
// (dwords per packet per lane, shipped 2), load look-ahead (blocks, shipped
// 1), 64-lane workgroups, the traffic-ceiling kernel (not a code),
// object-contiguous XCD map, LDS-staged inputs.
template <int W, int LW>
GfbFn pick_r_wg64(int r, bool acc) {
  static const GfbFn tbl[2][kMaxR] = {
      {&launch_gfb_t<W, 1, LW, false, kPF, false, 0, 64>, &launch_gfb_t<W, 2, LW, false, kPF, false, 0, 64>,
       &launch_gfb_t<W, 3, LW, false, kPF, false, 0, 64>, &launch_gfb_t<W, 4, LW, false, kPF, false, 0, 64>},
      {&launch_gfb_t<W, 1, LW, true, kPF, false, 0, 64>, &launch_gfb_t<W, 2, LW, true, kPF, false, 0, 64>,
       &launch_gfb_t<W, 3, LW, true, kPF, false, 0, 64>, &launch_gfb_t<W, 4, LW, true, kPF, false, 0, 64>}};
  return tbl[acc ? 1 : 0][r - 1];
}

// 16-byte lanes in 128-lane workgroups (2 KiB of every packet per tile, as
// the shipped 8-byte lanes in 256): a wave streams 1 KiB per packet instead
// of 512 B (tools/packet_ceiling.hip: the pattern reads 0.75-0.78 of peak
// against 0.66-0.72).
template <int W, int LW, int PF, int WG>
GfbFn pick_r_wg(int r, bool acc) {
  static const GfbFn tbl[2][kMaxR] = {
      {&launch_gfb_t<W, 1, LW, false, PF, false, 0, WG>, &launch_gfb_t<W, 2, LW, false, PF, false, 0, WG>,
       &launch_gfb_t<W, 3, LW, false, PF, false, 0, WG>, &launch_gfb_t<W, 4, LW, false, PF, false, 0, WG>},
      {&launch_gfb_t<W, 1, LW, true, PF, false, 0, WG>, &launch_gfb_t<W, 2, LW, true, PF, false, 0, WG>,
       &launch_gfb_t<W, 3, LW, true, PF, false, 0, WG>, &launch_gfb_t<W, 4, LW, true, PF, false, 0, WG>}};
  return tbl[acc ? 1 : 0][r - 1];
}

// At least `WAVES` waves per SIMD (the shipped form takes 132 VGPRs: 3).
template <int W, int LW, int PF, int WAVES>
GfbFn pick_r_waves(int r, bool acc) {
  static const GfbFn tbl[2][kMaxR] = {
      {&launch_gfb_t<W, 1, LW, false, PF, false, 0, kThreads, 0, WAVES>,
       &launch_gfb_t<W, 2, LW, false, PF, false, 0, kThreads, 0, WAVES>,
       &launch_gfb_t<W, 3, LW, false, PF, false, 0, kThreads, 0, WAVES>,
       &launch_gfb_t<W, 4, LW, false, PF, false, 0, kThreads, 0, WAVES>},
      {&launch_gfb_t<W, 1, LW, true, PF, false, 0, kThreads, 0, WAVES>,
       &launch_gfb_t<W, 2, LW, true, PF, false, 0, kThreads, 0, WAVES>,
       &launch_gfb_t<W, 3, LW, true, PF, false, 0, kThreads, 0, WAVES>,
       &launch_gfb_t<W, 4, LW, true, PF, false, 0, kThreads, 0, WAVES>}};
  return tbl[acc ? 1 : 0][r - 1];
}

GfbFn pick_measure8(int r, bool acc) {
  const Knobs& kn = knobs();
  // LEOEC_GFBIT_WAVES=4|5: the shipped form under a register cap
  if (kn.gfbit_waves == 4) return pick_r_waves<8, 2, kPF, 4>(r, acc);
  if (kn.gfbit_waves == 5) return pick_r_waves<8, 2, kPF, 5>(r, acc);
  if (kn.gfbit_wg == 64) return pick_r_wg64<8, 2>(r, acc);
  // LEOEC_GFBIT_WG=128: 16-byte lanes, next block's loads in flight
  // (LEOEC_GFBIT_PF=0: load-then-compute; the round-2 abort of this form,
  // profiles/r02_v15_cauchy_lw16_pf0_abort.log, is diagnosed in DESIGN.md)
  if (kn.gfbit_wg == 128)
    return kn.gfbit_pf == 0 ? pick_r_wg<8, 4, 0, 128>(r, acc) : pick_r_wg<8, 4, 1, 128>(r, acc);
  const int lw = kn.gfbit_lw;
  if (kn.gfbit_ceil && r == 4 && !acc) return &launch_gfb_t<8, 4, 2, false, kPF, true>;
  if (kn.gfbit_xmap == 1 && r == 4 && !acc)
    return &launch_gfb_t<8, 4, 2, false, kPF, false, 0, kThreads, 1>;
  if (kn.gfbit_lds == 1) {
    static const GfbFn tbl[2][kMaxR] = {
        {&launch_gfb_lds_t<8, 1, false>, &launch_gfb_lds_t<8, 2, false>,
         &launch_gfb_lds_t<8, 3, false>, &launch_gfb_lds_t<8, 4, false>},
        {&launch_gfb_lds_t<8, 1, true>, &launch_gfb_lds_t<8, 2, true>,
         &launch_gfb_lds_t<8, 3, true>, &launch_gfb_lds_t<8, 4, true>}};
    return tbl[acc ? 1 : 0][r - 1];
  }
  const int pf = kn.gfbit_pf;
  if (pf == 0) {
    if (lw == 1) return pick_r<8, 1, 0>(r, acc);
    if (lw == 4) return pick_r<8, 4, 0>(r, acc);
    return pick_r<8, 2, 0>(r, acc);
  }
  if (pf == 2) {
    if (lw == 1) return pick_r<8, 1, 2>(r, acc);
    return pick_r<8, 2, 2>(r, acc);
  }
  if (pf == 3) {
    if (lw == 1) return pick_r<8, 1, 3>(r, acc);
    return pick_r<8, 2, 3>(r, acc);
  }
  if (lw == 1) return pick_r<8, 1>(r, acc);
  if (lw == 4) return pick_r<8, 4>(r, acc);
  return pick_r<8, 2>(r, acc);
}

// LEOEC_GFBIT_PF = blocks in flight (1..3), LEOEC_GFBIT_WG = 64 | 128 | 256,
// LEOEC_GFBIT_WAVES = 2: at most 256 VGPRs (default: one wave per SIMD
// allowed).  (The MASK = 1 form spills at every look-ahead: 512 VGPRs + 537
// spilled, so it has no launch entry.)
GfbFn pick_gfbk() {
  const Knobs& kn = knobs();
  const int la = kn.gfbit_pf < 1 ? 1 : kn.gfbit_pf > 3 ? 3 : kn.gfbit_pf;
  if (kn.gfbit_waves == 2) {
    if (kn.gfbit_wg == 64) return la == 1 ? &launch_gfbk_t<1, 64, false, 2> : &launch_gfbk_t<2, 64, false, 2>;
    return la == 1 ? &launch_gfbk_t<1, 128, false, 2> : &launch_gfbk_t<2, 128, false, 2>;
  }
  if (kn.gfbit_wg == 64)
    return la == 1 ? &launch_gfbk_t<1, 64, false, 1> : la == 2 ? &launch_gfbk_t<2, 64, false, 1> : &launch_gfbk_t<3, 64, false, 1>;
  if (kn.gfbit_wg == 256) return la == 1 ? &launch_gfbk_t<1, 256, false, 1> : &launch_gfbk_t<2, 256, false, 1>;
  return la == 1 ? &launch_gfbk_t<1, 128, false, 1> : la == 2 ? &launch_gfbk_t<2, 128, false, 1> : &launch_gfbk_t<3, 128, false, 1>;
}

GfbFn pick2(int w, int r, bool acc) {
  switch (w) {
    case 8: return measure2<8>(r, acc);
    case 2: return measure2<2>(r, acc);
    case 3: return measure2<3>(r, acc);
    case 4: return measure2<4>(r, acc);
    case 5: return measure2<5>(r, acc);
    case 6: return measure2<6>(r, acc);
    case 7: return measure2<7>(r, acc);
    case 9: return measure2<9>(r, acc);
    case 10: return measure2<10>(r, acc);
    case 11: return measure2<11>(r, acc);
    case 12: return measure2<12>(r, acc);
    case 13: return measure2<13>(r, acc);
    case 14: return measure2<14>(r, acc);
    case 15: return measure2<15>(r, acc);
    case 16: return measure2<16>(r, acc);
    default: return nullptr;
  }
}
}  // namespace

GfbFn pick_measure(const GfBitApply& p, int w, int r, bool acc, int nk, bool big) {
  // LEOEC_GFBIT_FORM=1: gfb2_apply (LEOEC_GFBIT_LW=1: 4 bytes per lane per
  // packet at w = 8; LEOEC_GFBIT_PF=1: its prefetching loop)
  // LEOEC_GFBIT_FORM=2: gfbx_apply where it applies (w = 8, 4 rows, one input
  // chunk, no accumulation), the shipped kernel otherwise
  if (knobs().gfbit_form == 2 && w == 8 && r == 4 && !acc && nk <= kMaxK)
    return &launch_gfbx_8;
  if (knobs().gfbit_form == 3 && gfba_applies(p, w, acc, nk)) return pick_gfba_knobs(r);
  // LEOEC_GFBIT_FORM=5: gfbk_apply where it applies (w = 8, K = 10, 4 rows,
  // no accumulation), the shipped kernel otherwise
  if (knobs().gfbit_form == 5 && w == 8 && r == 4 && !acc && nk == 10) return pick_gfbk();
  if (knobs().gfbit_form == 1) {
    // LEOEC_GFBIT_WG=128: 16-byte lanes in 128-lane workgroups, next block in flight
    if (w == 8 && knobs().gfbit_wg == 128) return pick_r2<8, 4, 1, 128>(r, acc);
    if (w == 8 && knobs().gfbit_lw == 1) return pick_r2<8, 1>(r, acc);
    if (w == 8 && knobs().gfbit_pf == 1) return pick_r2<8, 2, 1>(r, acc);
    return pick2(w, r, acc);
  }
  // (a launch above the gfbk threshold without an explicit form: gfbk_apply,
  // as in the product; LEOEC_GFBK_MIN_MIB moves the threshold)
  if (w == 8 && !big) return pick_measure8(r, acc);
  return nullptr;
}

}  // namespace gfbit_detail
}  // namespace leoec
