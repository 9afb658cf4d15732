// gfbit_inst.hip — launches of the packet-bitsliced GF(2^w) kernel
// (kernels_impl.hpp gfbit_apply) for w = 2..16, R <= 4 outputs per launch,
// inputs beyond 16 folded in by accumulating launches.
#include <utility>

#include "kernels_impl.hpp"
#include "knobs.hpp"

namespace leoec {

using namespace detail;

namespace {

using GfbFn = int (*)(const GfBitApply&, int r0, int j0, int nk, uint64_t o0, uint64_t no,
                      hipStream_t);

template <int W, int R, int LW, bool ACC, int PF, bool CEIL = false, int KR = 0,
          int WG = kThreads, int XMAP = 0>
int launch_gfb_t(const GfBitApply& p, int r0, int j0, int nk, uint64_t o0, uint64_t no,
                 hipStream_t s) {
  GfbArgs<R> a;
  a.K = nk;
  a.ps = (uint32_t)(p.block_size / (uint64_t)W);
  constexpr uint32_t tb = WG * 4u * LW;
  a.tiles = (a.ps + tb - 1) / tb;
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
  hipLaunchKernelGGL((gfbit_apply<W, R, LW, ACC, PF, CEIL, KR, WG, XMAP>),
                     dim3((uint32_t)(no * a.tiles)), dim3(WG), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

constexpr int kPF = 1;  // blocks of load look-ahead (kernels_impl.hpp gfbit_apply)

#ifdef LEOEC_MEASURE
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
#endif  // LEOEC_MEASURE

template <int W, int LW, int PF = kPF>
GfbFn pick_r(int r, bool acc) {
  static const GfbFn tbl[2][kMaxR] = {
      {&launch_gfb_t<W, 1, LW, false, PF>, &launch_gfb_t<W, 2, LW, false, PF>,
       &launch_gfb_t<W, 3, LW, false, PF>, &launch_gfb_t<W, 4, LW, false, PF>},
      {&launch_gfb_t<W, 1, LW, true, PF>, &launch_gfb_t<W, 2, LW, true, PF>,
       &launch_gfb_t<W, 3, LW, true, PF>, &launch_gfb_t<W, 4, LW, true, PF>}};
  return tbl[acc ? 1 : 0][r - 1];
}

#ifdef LEOEC_MEASURE
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

GfbFn pick_measure8(int r, bool acc) {
  const Knobs& kn = knobs();
  if (kn.gfbit_wg == 64) return pick_r_wg64<8, 2>(r, acc);
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
#endif  // LEOEC_MEASURE

GfbFn pick(int w, int r, bool acc, int nk) {
  (void)nk;
#ifdef LEOEC_MEASURE
  if (w == 8) return pick_measure8(r, acc);
#endif
  switch (w) {
    case 8: return pick_r<8, 2>(r, acc);
    case 2: return pick_r<2, 2>(r, acc);
    case 3: return pick_r<3, 2>(r, acc);
    case 4: return pick_r<4, 2>(r, acc);
    case 5: return pick_r<5, 2>(r, acc);
    case 6: return pick_r<6, 2>(r, acc);
    case 7: return pick_r<7, 2>(r, acc);
    case 9: return pick_r<9, 2>(r, acc);
    case 10: return pick_r<10, 2>(r, acc);
    case 11: return pick_r<11, 2>(r, acc);
    case 12: return pick_r<12, 1>(r, acc);
    case 13: return pick_r<13, 1>(r, acc);
    case 14: return pick_r<14, 1>(r, acc);
    case 15: return pick_r<15, 1>(r, acc);
    case 16: return pick_r<16, 1>(r, acc);
    default: return nullptr;
  }
}

}  // namespace

bool gfbit_supported(int w) { return w >= 2 && w <= 16; }

int launch(const GfBitApply& p, hipStream_t s) {
  const int w = p.w;
  if (!gfbit_supported(w) || p.K <= 0 || p.R <= 0 || (int)p.in.size() != p.K ||
      (int)p.out.size() != p.R || p.coef.size() != (size_t)p.K * p.R)
    return LEOEC_E_ARG;
  if (p.block_size == 0 || p.nobj == 0) return LEOEC_OK;
  if (p.block_size % ((uint64_t)16 * w) || p.block_size >= (1ull << 32)) return LEOEC_E_BAD_SIZE;
  for (const Shard& sh : p.in)
    if (((uintptr_t)sh.base & 15u) || (sh.stride & 15u)) return LEOEC_E_ARG;
  for (const Shard& sh : p.out)
    if (((uintptr_t)sh.base & 15u) || (sh.stride & 15u)) return LEOEC_E_ARG;
  const uint64_t ps = p.block_size / (uint64_t)w;
  const uint64_t tiles = (ps + 1023) / 1024;  // smallest lane width -> most tiles
  const uint64_t max_obj = (uint64_t)0x7FFFFFFF / tiles;
  for (uint64_t o0 = 0; o0 < p.nobj; o0 += max_obj) {
    const uint64_t no = (p.nobj - o0 < max_obj) ? p.nobj - o0 : max_obj;
    for (int r0 = 0; r0 < p.R; r0 += kMaxR) {
      const int nr = (p.R - r0 < kMaxR) ? p.R - r0 : kMaxR;
      for (int j0 = 0; j0 < p.K; j0 += kMaxK) {
        const int nk = (p.K - j0 < kMaxK) ? p.K - j0 : kMaxK;
        const int rc = pick(w, nr, j0 > 0, nk)(p, r0, j0, nk, o0, no, s);
        if (rc) return rc;
      }
    }
  }
  return LEOEC_OK;
}

}  // namespace leoec
