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
