// gf8_exp.hip — measurement variants of gf8_apply<10, 4> (the RS(10,4,8)
// headline shape), selected with LEOEC_GF8_VARIANT=<n> for A/B runs in one
// process (tools/kvariants.py).  Variant 1 is the shipped configuration.
#include "kernels_impl.hpp"

namespace leoec {
namespace detail {

ChunkFn gf8_variant(int v) {
  //                            K   R  ACC    CPT  NT     BRANCHY COPY   PIPE
  switch (v) {
    case 1: return &launch_gf8_t<10, 4, false, 1, true, -1, false, false>;  // shipped
    case 2: return &launch_gf8_t<10, 4, false, 2, true, -1, false, false>;
    case 3: return &launch_gf8_t<10, 4, false, 1, true, 1, false, false>;   // always branchy
    case 5: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false>;   // always paired
    case 7: return &launch_gf8_t<10, 4, false, 1, true, 1, true, false>;    // copy-xor
    case 12: return &launch_gf8_t<10, 4, false, 1, false, -1, false, false>;  // no nt
    case 13: return &launch_gf8_t<10, 4, false, 1, true, -1, false, true>;  // persistent prefetch
    case 14: return &launch_gf8_t<10, 4, false, 1, true, 1, true, true>;    // copy-xor persistent
    default: return nullptr;
  }
}

}  // namespace detail
}  // namespace leoec
