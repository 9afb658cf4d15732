// gf8_exp.hip — measurement variants of gf8_apply<10, 4> (the RS(10,4,8)
// headline shape), selected with LEOEC_GF8_VARIANT=<n> for A/B runs in one
// process (tools/kvariants.py).  Variant 1 is the shipped configuration.
#include "kernels_impl.hpp"

namespace leoec {
namespace detail {

ChunkFn gf8_variant(int v) {
  //                            K   R  ACC    CPT  NT     BRANCHY COPY
  switch (v) {
    case 1: return &launch_gf8_t<10, 4, false, 1, true, true, false>;   // shipped
    case 11: return &launch_gf8_t<10, 4, false, 1, true, false, false>;  // nt + branchfree
    case 12: return &launch_gf8_t<10, 4, false, 1, false, true, false>;  // no nt
    case 2: return &launch_gf8_t<10, 4, false, 2, false, true, false>;
    case 3: return &launch_gf8_t<10, 4, false, 1, true, true, false>;
    case 4: return &launch_gf8_t<10, 4, false, 2, true, true, false>;
    case 5: return &launch_gf8_t<10, 4, false, 1, false, false, false>;
    case 6: return &launch_gf8_t<10, 4, false, 1, false, true, true>;
    case 7: return &launch_gf8_t<10, 4, false, 1, true, true, true>;
    case 8: return &launch_gf8_t<10, 4, false, 2, false, false, false>;
    case 9: return &launch_gf8_t<10, 4, false, 4, false, true, false>;
    case 10: return &launch_gf8_t<10, 4, false, 2, false, true, true>;
    default: return nullptr;
  }
}

}  // namespace detail
}  // namespace leoec
