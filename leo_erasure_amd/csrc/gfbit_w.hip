// gfbit_w.hip — the packet-bitsliced kernel's launch tables for one field
// width, compiled once per w = 2..16 (-DLEOEC_GFBIT_W=w) so the instances of
// gfbit_apply (and, in the measurement build, gfb2_apply) compile in
// parallel.  Lane width: 2 dwords per packet up to w = 11, 1 from w = 12
// (packets of bs / w bytes, bs a multiple of 16 w).
#include "gfbit_impl.hpp"

#ifndef LEOEC_GFBIT_W
#error "compile with -DLEOEC_GFBIT_W=<2..16>"
#endif

namespace leoec {
namespace gfbit_detail {

constexpr int kW = LEOEC_GFBIT_W;
constexpr int kLW = kW >= 12 ? 1 : 2;

template <>
GfbFn shipped<kW>(int r, bool acc) {
  return pick_r<kW, kLW>(r, acc);
}

#ifdef LEOEC_MEASURE
template <>
GfbFn measure2<kW>(int r, bool acc) {
  return pick_r2<kW, kLW>(r, acc);
}
#endif

}  // namespace gfbit_detail
}  // namespace leoec
