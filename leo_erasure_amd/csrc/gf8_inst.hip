// gf8_inst.hip — GF(2^8) kernel instances for one input count K (compiled
// once per K = 1..16 with -DLEOEC_GF8_K=K; see kernels_impl.hpp).
#include "kernels_impl.hpp"

#ifndef LEOEC_GF8_K
#error "compile with -DLEOEC_GF8_K=<1..16>"
#endif

namespace leoec {
namespace detail {

template <>
ChunkFn gf8_launcher<LEOEC_GF8_K>(int r, bool acc) {
  constexpr int K = LEOEC_GF8_K;
  static const ChunkFn tbl[2][kMaxR] = {
      {&launch_gf8_t<K, 1, false>, &launch_gf8_t<K, 2, false>, &launch_gf8_t<K, 3, false>,
       &launch_gf8_t<K, 4, false>},
      {&launch_gf8_t<K, 1, true>, &launch_gf8_t<K, 2, true>, &launch_gf8_t<K, 3, true>,
       &launch_gf8_t<K, 4, true>}};
  return tbl[acc ? 1 : 0][r - 1];
}

}  // namespace detail
}  // namespace leoec
