// lib_inst.hip — the liberation kernels with branch-free loads (libb_apply,
// libb_dec_apply, kernels_impl.hpp) for one w, every k = 1..w compiled in
// (the block count is a template argument: a run-time k put a uniform branch
// between blocks, and the compiler sank the next block's loads below it),
// compiled once per w = 3, 5, 7, 11, 13 (-DLEOEC_LIB_W=w) so the instances
// build in parallel.  The measurement build adds look-ahead 4 / 8 and the
// other lane count for the A/B configurations (k = 4, 7 at w = 7; k = 10 at
// w = 11; k = w at w = 5, 13), and the syndrome kernel's block form
// (look-ahead 0: absent shards skipped).
#include <utility>

#include "kernels_impl.hpp"

#ifndef LEOEC_LIB_W
#error "compile with -DLEOEC_LIB_W=<3|5|7|11|13>"
#endif

namespace leoec {
namespace detail {

namespace {

constexpr int kW = LEOEC_LIB_W;
#ifdef LEOEC_MEASURE
constexpr bool kMeasureBuildTU = true;
#else
constexpr bool kMeasureBuildTU = false;
#endif

// libb_apply is shipped for w >= kLibbEncMinW only; the measurement build
// has it at every w (LEOEC_LIB_BUF=1 forces it, A/B and parity)
constexpr bool kEncBuilt = kMeasureBuildTU || kW >= kLibbEncMinW;

template <std::size_t... I>
LibbEnc enc_shipped(std::index_sequence<I...>, int k) {
  if constexpr (kEncBuilt) {
    static const LibbEnc tbl[] = {
        {&libb_apply<kW, (int)I + 1, kLibbEncLA, kLibbEncTW>, (uint32_t)kLibbEncTW}...};
    return tbl[k - 1];
  } else {
    (void)k;
    return {nullptr, 0};
  }
}
template <std::size_t... I>
LibbDec dec_shipped(std::index_sequence<I...>, int k) {
  static const LibbDec tbl[] = {
      {&libb_dec_apply<kW, (int)I + 1, libb_dec_la(kW, (int)I + 1), kLibbDecTW>,
       (uint32_t)kLibbDecTW}...};
  return tbl[k - 1];
}

#ifdef LEOEC_MEASURE
template <int K>
LibbEnc enc_form(int la, int tw) {
  if (tw == 256) {
    if (la == 4) return {&libb_apply<kW, K, 4, 256>, 256u};
    if (la == 8) return {&libb_apply<kW, K, 8, 256>, 256u};
    return {&libb_apply<kW, K, 2, 256>, 256u};
  }
  if (la == 4) return {&libb_apply<kW, K, 4, 64>, 64u};
  if (la == 8) return {&libb_apply<kW, K, 8, 64>, 64u};
  return {&libb_apply<kW, K, 2, 64>, 64u};
}
template <int K>
LibbDec dec_form(int la, int tw) {
  if (tw == 64) {
    if (la == 0) return {&libb_dec_apply<kW, K, 0, 64>, 64u};  // block form
    if (la == 4) return {&libb_dec_apply<kW, K, 4, 64>, 64u};
    if (la == 8) return {&libb_dec_apply<kW, K, 8, 64>, 64u};
    return {&libb_dec_apply<kW, K, 2, 64>, 64u};
  }
  if (la == 0) return {&libb_dec_apply<kW, K, 0, 256>, 256u};
  if (la == 4) return {&libb_dec_apply<kW, K, 4, 256>, 256u};
  if (la == 8) return {&libb_dec_apply<kW, K, 8, 256>, 256u};
  return {&libb_dec_apply<kW, K, 2, 256>, 256u};
}
#endif

}  // namespace

template <>
LibbEnc libb_enc_pick<kW>(int k, int la, int tw) {
  if (k < 1 || k > kW) return {nullptr, 0};
#ifdef LEOEC_MEASURE
  if (la != kLibbEncLA || tw != kLibbEncTW) {
    if constexpr (kW == 7) {
      if (k == 4) return enc_form<4>(la, tw);
      if (k == 7) return enc_form<7>(la, tw);
    }
    if constexpr (kW == 11) {
      if (k == 10) return enc_form<10>(la, tw);
    }
    if constexpr (kW == 5) {
      if (k == 5) return enc_form<5>(la, tw);
    }
    if constexpr (kW == 13) {
      if (k == 13) return enc_form<13>(la, tw);
    }
  }
#endif
  (void)la;
  (void)tw;
  return enc_shipped(std::make_index_sequence<kW>{}, k);
}

template <>
LibbDec libb_dec_pick<kW>(int k, int la, int tw) {
  if (k < 1 || k > kW) return {nullptr, 0};
#ifdef LEOEC_MEASURE
  if (la != libb_dec_la(kW, k) || tw != kLibbDecTW) {
    if constexpr (kW == 7) {
      if (k == 4) return dec_form<4>(la, tw);
      if (k == 7) return dec_form<7>(la, tw);
    }
    if constexpr (kW == 11) {
      if (k == 10) return dec_form<10>(la, tw);
    }
    if constexpr (kW == 5) {
      if (k == 5) return dec_form<5>(la, tw);
    }
    if constexpr (kW == 13) {
      if (k == 13) return dec_form<13>(la, tw);
    }
  }
#endif
  (void)la;
  (void)tw;
  return dec_shipped(std::make_index_sequence<kW>{}, k);
}

}  // namespace detail
}  // namespace leoec
