// gfbit_inst.hip — the packet-bitsliced GF(2^w) kernel for w = 2..16
// (cauchyrs; kernels_impl.hpp gfbit_apply for the arithmetic), R <= 4
// outputs per launch, inputs beyond 16 folded in by accumulating launches.
//
// gfbit_apply (kernels_impl.hpp) is shipped, and gfbk_apply (gfbit_impl.hpp)
// for launches of at least kGfbkMinBytes of the (w = 8, K = 10, 4 rows)
// shape; this TU holds their launch dispatch (and gfbk's instance).  The
// measurement forms (gfb2_apply, gfbx_apply, gfba_apply, the lane-width /
// look-ahead / register-cap / LDS variants) live in gfbit_measure.hip,
// compiled into the measurement library only.
#include <utility>

#include "gfbit_impl.hpp"

namespace leoec {

using namespace detail;

namespace {

using namespace gfbit_detail;

GfbFn pick(const GfBitApply& p, int w, int r, bool acc, int nk, uint64_t no) {
  // large cauchyrs(k = 10, w = 8)-shaped launches: gfbk_apply (gfbit_impl.hpp)
  const bool big = gfbk_pays(p, r, acc, nk, no);
#ifdef LEOEC_MEASURE
  // the measurement forms (gfbit_measure.hip) where LEOEC_GFBIT_* selects one
  if (GfbFn f = pick_measure(p, w, r, acc, nk, big)) return f;
#endif
  if (big) return &launch_gfbk_t<3, 64, false, 1>;
  switch (w) {
    case 8: return shipped<8>(r, acc);
    case 2: return shipped<2>(r, acc);
    case 3: return shipped<3>(r, acc);
    case 4: return shipped<4>(r, acc);
    case 5: return shipped<5>(r, acc);
    case 6: return shipped<6>(r, acc);
    case 7: return shipped<7>(r, acc);
    case 9: return shipped<9>(r, acc);
    case 10: return shipped<10>(r, acc);
    case 11: return shipped<11>(r, acc);
    case 12: return shipped<12>(r, acc);
    case 13: return shipped<13>(r, acc);
    case 14: return shipped<14>(r, acc);
    case 15: return shipped<15>(r, acc);
    case 16: return shipped<16>(r, acc);
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
  {
    int rc = LEOEC_OK;
    if (launch_cbm(p, s, &rc)) return rc;
  }
  const uint64_t ps = p.block_size / (uint64_t)w;
  // the narrowest tile of any form (64 lanes x 8 bytes, LEOEC_GFBIT_WG=64)
  // bounds the grid: every form's tile count is at most this
  const uint64_t tiles = (ps + 511) / 512;
  const uint64_t max_obj = (uint64_t)0x7FFFFFFF / tiles;
  for (uint64_t o0 = 0; o0 < p.nobj; o0 += max_obj) {
    const uint64_t no = (p.nobj - o0 < max_obj) ? p.nobj - o0 : max_obj;
    for (int r0 = 0; r0 < p.R; r0 += kMaxR) {
      const int nr = (p.R - r0 < kMaxR) ? p.R - r0 : kMaxR;
      for (int j0 = 0; j0 < p.K; j0 += kMaxK) {
        const int nk = (p.K - j0 < kMaxK) ? p.K - j0 : kMaxK;
        const int rc = pick(p, w, nr, j0 > 0, nk, no)(p, r0, j0, nk, o0, no, s);
        if (rc) return rc;
      }
    }
  }
  return LEOEC_OK;
}

}  // namespace leoec
