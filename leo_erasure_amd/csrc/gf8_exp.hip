// gf8_exp.hip — measurement variants of gf8_apply<10, 4> (the RS(10,4,8)
// headline shape), selected with LEOEC_GF8_VARIANT=<n> for A/B runs in one
// process (tools/kvariants.py).  Variant 1 is the shipped configuration.
#include "kernels_impl.hpp"

namespace leoec {
namespace detail {

ChunkFn gf8_variant(int v) {
  //                             K   R  ACC    CPT NT    BR  COPY   PIPE   LDS
  switch (v) {
    case 1: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true>;   // shipped
    case 2: return &launch_gf8_t<10, 4, false, 2, true, 0, false, false, true>;   // cpt2
    case 3: return &launch_gf8_t<10, 4, false, 1, true, 1, false, false, false>;  // branchy sgpr
    case 4: return &launch_gf8_t<10, 4, false, 1, true, 1, false, false, true>;   // branchy lds
    case 5: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, false>;  // paired sgpr
    case 7: return &launch_gf8_t<10, 4, false, 1, true, 1, true, false, false>;   // copy-xor
    case 12: return &launch_gf8_t<10, 4, false, 1, false, 0, false, false, true>; // no nt
    case 15: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5>;  // >=5 waves
    case 16: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 6>;  // >=6 waves
    case 17: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 8>;  // 8 waves
    case 20: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 512>;
    case 21: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 1>;
    case 22: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 512, 1>;
    case 23: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 1024>;
    case 24: return &launch_gf8_t<10, 4, false, 1, true, 1, true, false, false, 5, 256, 1>;  // copy xmap
    case 25: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 64>;   // wg64
    case 26: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 128>;  // wg128
    case 27: return &launch_gf8_t<10, 4, false, 1, true, 1, true, false, false, 5, 64>;   // copy wg64
    case 28: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 4, 64>;   // wg64 >=4 waves
    case 30: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 2, true>;  // buffer ld/st
    case 31: return &launch_gf8_t<10, 4, false, 1, true, 1, true, false, false, 5, 256, 2, true>;  // copy buffer
    case 32: return &launch_gf8_t<10, 4, false, 1, true, -1, false, false, true, 5, 256, 2, true>; // buffer, auto branchy
    case 33: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 2, false, true>;  // row 0 / column 0 of ones folded
    case 34: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 2>;  // xcd_obj_map always
    case 35: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 64, 0, true>;  // buffer ld/st wg64, run-time tile map
    case 36: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 0, false, false, true>;  // loads before LDS staging
    case 37: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 5, 256, 0, true, false, true>;   // + buffer ld/st
    case 29: return &launch_gf8_t<10, 4, false, 1, true, 0, false, false, true, 6, 64>;   // wg64 >=6 waves
    default: return nullptr;
  }
}

}  // namespace detail
}  // namespace leoec
