// kernels.hip — dispatch of GfApply / BitApply plans onto the gfx950 kernels
// of kernels_impl.hpp (w = 16/32 and bitmatrix instances live here; GF(2^8)
// instances in gf8_inst.hip).
#include <utility>

#include "kernels_impl.hpp"
#include "knobs.hpp"

namespace leoec {

using namespace detail;

namespace {

bool shards_ok(const std::vector<Shard>& v) {
  for (const Shard& s : v)
    if (((uintptr_t)s.base & 15u) || (s.stride & 15u)) return false;
  return true;
}

template <std::size_t... I>
ChunkFn gf8_pick(std::index_sequence<I...>, int k, int r, bool acc) {
  static ChunkFn (*const sel[])(int, bool) = {&gf8_launcher<(int)I + 1>...};
  return sel[k - 1](r, acc);
}

#ifdef LEOEC_MEASURE
ChunkFn gf16_pick(int r, bool acc) {
  static const ChunkFn tbl[2][kMaxR] = {
      {&launch_gf16_t<1, false>, &launch_gf16_t<2, false>, &launch_gf16_t<3, false>,
       &launch_gf16_t<4, false>},
      {&launch_gf16_t<1, true>, &launch_gf16_t<2, true>, &launch_gf16_t<3, true>,
       &launch_gf16_t<4, true>}};
  return tbl[acc ? 1 : 0][r - 1];
}

#endif  // LEOEC_MEASURE

// Knobs::gfw_form selects the w = 16 / 32 kernel (measurement build):
//   3 bitsliced planes (gfs_apply, gfs_inst.hip; shipped)
//   0 byte-plane v_perm (gfp_apply, shipped in round 1)
//   1 w=16: 2-bit-field v_perm (gf16_apply); w=32: shift-and-add
//   2 shift-and-add (gfw_apply)
// Knobs::gfp_cpt = 1|2 sets gfp_apply's 16-byte columns per lane (2 shipped).
#ifdef LEOEC_MEASURE
template <int W>
ChunkFn gfp_pick(int r, bool acc, int cpt) {
  static const ChunkFn tbl[2][2][kMaxR] = {
      {{&launch_gfp_t<W, 1, false, 1>, &launch_gfp_t<W, 2, false, 1>,
        &launch_gfp_t<W, 3, false, 1>, &launch_gfp_t<W, 4, false, 1>},
       {&launch_gfp_t<W, 1, true, 1>, &launch_gfp_t<W, 2, true, 1>, &launch_gfp_t<W, 3, true, 1>,
        &launch_gfp_t<W, 4, true, 1>}},
      {{&launch_gfp_t<W, 1, false, 2>, &launch_gfp_t<W, 2, false, 2>,
        &launch_gfp_t<W, 3, false, 2>, &launch_gfp_t<W, 4, false, 2>},
       {&launch_gfp_t<W, 1, true, 2>, &launch_gfp_t<W, 2, true, 2>, &launch_gfp_t<W, 3, true, 2>,
        &launch_gfp_t<W, 4, true, 2>}}};
  return tbl[cpt == 2 ? 1 : 0][acc ? 1 : 0][r - 1];
}

template <int W>
ChunkFn gfw_pick(int r, bool acc) {
  static const ChunkFn tbl[2][kMaxR] = {
      {&launch_gfw_t<W, 1, false>, &launch_gfw_t<W, 2, false>, &launch_gfw_t<W, 3, false>,
       &launch_gfw_t<W, 4, false>},
      {&launch_gfw_t<W, 1, true>, &launch_gfw_t<W, 2, true>, &launch_gfw_t<W, 3, true>,
       &launch_gfw_t<W, 4, true>}};
  return tbl[acc ? 1 : 0][r - 1];
}

#endif  // LEOEC_MEASURE

// Knobs::gf8_variant = <n> selects a measurement variant of gf8_apply<10,4>
// (tools/kvariants.py); 0 = the shipped kernel.
// Knobs::bit_form selects the bitmatrix kernel form for measurements:
//   0 masked, no look-ahead        1 masked, 1 packet ahead
//   2 branchy, no look-ahead       3 branchy, 1 packet ahead
//   4/5/6 masked, 2/3/5 packets ahead (4 = shipped)
//   7 as 4, with all tiles of an object on one XCD
//   8 as 4, output packets padded to 8 / 16 / 32 (4 pads to even)
//   9 as 4, objects interleaved over the XCDs (xcd_obj_map)
// Measured on liberation(7,2,7): masked beats branchy (the scalar branches
// cost more than the masked xors they save); look-ahead depth see DESIGN.md.
using BitFn = void (*)(const detail::BitArgs);

#ifdef LEOEC_MEASURE
template <int RO, bool ACC>
BitFn bit_kernel_f(int form) {
  switch (form) {
    case 0: return &detail::bit_apply<RO, ACC, false, 0>;
    case 1: return &detail::bit_apply<RO, ACC, false, 1>;
    case 2: return &detail::bit_apply<RO, ACC, true, 0>;
    case 3: return &detail::bit_apply<RO, ACC, true, 1>;
    case 5: return &detail::bit_apply<RO, ACC, false, 3>;
    case 6: return &detail::bit_apply<RO, ACC, false, 5>;
    case 7: return &detail::bit_apply<RO, ACC, false, 2, 1>;
    case 9: return &detail::bit_apply<RO, ACC, false, 2, 2>;
    default: return &detail::bit_apply<RO, ACC, false, 2>;
  }
}

BitFn bit_kernel(int ro, bool acc, int form) {
  if (ro == 8) return acc ? bit_kernel_f<8, true>(form) : bit_kernel_f<8, false>(form);
  if (ro == 16) return acc ? bit_kernel_f<16, true>(form) : bit_kernel_f<16, false>(form);
  return acc ? bit_kernel_f<32, true>(form) : bit_kernel_f<32, false>(form);
}
#endif  // LEOEC_MEASURE

// Shipped form with the output-packet count rounded up to even only (2..32):
// liberation(k,2,w) has 2w output packets (14 at w=7, 22 at w=11), which the
// {8,16,32} instances pad by up to 45 % of masked xors.
template <std::size_t... I>
BitFn bit_kernel_even(std::index_sequence<I...>, int rp, bool acc) {
  static const BitFn tbl[2][sizeof...(I)] = {
      {&detail::bit_apply<2 * ((int)I + 1), false, false, 2>...},
      {&detail::bit_apply<2 * ((int)I + 1), true, false, 2>...}};
  return tbl[acc ? 1 : 0][(rp + 1) / 2 - 1];
}

// True when the plan is exactly a liberation encode bitmatrix (the structure
// lib_apply<W> compiles in, kernels_impl.hpp): RB = 2, KB <= w, and bit
// (o, j*w + x) set iff o = x (P), or o = w + (x - j) mod w (Q), or, for
// j > 0, o = w + y with y = j (w-1)/2 mod w and x = (y + j - 1) mod w.
bool is_liberation_encode(const BitApply& p) {
  const int w = p.w, k = p.KB;
  if (p.RB != 2 || k > w || k > kMaxK) return false;
  const size_t cols = (size_t)k * w;
  for (int j = 0; j < k; ++j) {
    const int y = (j * ((w - 1) / 2)) % w;
    for (int x = 0; x < w; ++x)
      for (int o = 0; o < 2 * w; ++o) {
        bool want = (o == x) || (o == w + (x - j + w) % w);
        if (j > 0 && o == w + y && x == (y + j - 1) % w) want = true;
        if ((p.bits[(size_t)o * cols + (size_t)j * w + x] != 0) != want) return false;
      }
  }
  return true;
}

// Knobs::lib_form = 0 routes liberation encodes through the generic masked
// bitmatrix kernel (A/B and parity of both forms); 1 = lib_apply (shipped).
// Knobs::lib_la = 2|4|8 sets lib_apply's packet look-ahead (measurement
// build; shipped 2: profiles/r01_v13_ab_lib_la.log, best or within 1 % of
// best for w = 5..13).
// lib_apply runs 64-lane workgroups (1 KiB of every packet per tile):
// liberation 1 MiB encode (7,2,7) 0.682 -> 0.686, (10,2,11) 0.694 -> 0.700,
// (4,2,7) 0.662 -> 0.689 against 256 lanes (profiles/r02_v22_ab_lib_wg_*.log).
// Knobs::lib_wg = 256 (measurement build) restores the 256-lane form, which
// the look-ahead variants (lib_la 4 / 8) also use.
using LibFn = void (*)(const detail::LibArgs);
constexpr uint32_t kLibLanes = 64;
uint32_t lib_lanes() {
  if (!kMeasureBuild) return kLibLanes;
  const Knobs& k = knobs();
  return (k.lib_wg == 256 || k.lib_la != 2) ? (uint32_t)kThreads : kLibLanes;
}
template <int W>
LibFn lib_kernel_w(int la) {
  // (the product ships libb_apply from w = kLibbEncMinW: no lib_apply there)
  if constexpr (!kMeasureBuild && W >= kLibbEncMinW) return nullptr;
#ifdef LEOEC_MEASURE
  if (la == 4) return &detail::lib_apply<W, 4>;  // 256 lanes (lib_lanes())
  if (la == 8) return &detail::lib_apply<W, 8>;
  if (lib_lanes() == (uint32_t)kThreads) return &detail::lib_apply<W, 2>;
#endif
  (void)la;
  return &detail::lib_apply<W, 2, kLibLanes>;
}
// Knobs::lib_xmap = 0 (A/B): workgroup ids in dispatch order instead of the
// object-interleaved XCD map (xcd_obj_map, kernels_impl.hpp) that the
// launchers use for objects of at most kObjMapMaxTiles tiles
bool obj_map(uint32_t tiles) { return tiles <= kObjMapMaxTiles && knobs().lib_xmap != 0; }
LibFn lib_kernel(int w) {
  const int la = knobs().lib_la;
  switch (w) {
    case 3: return lib_kernel_w<3>(la);
    case 5: return lib_kernel_w<5>(la);
    case 7: return lib_kernel_w<7>(la);
    case 11: return lib_kernel_w<11>(la);
    case 13: return lib_kernel_w<13>(la);
    default: return nullptr;
  }
}

// Knobs::lib_buf: the branch-free forms (libb_apply / libb_dec_apply,
// lib_inst.hip), look-ahead lib_la / lib_dec_la and lib_wg / lib_dec_wg
// lanes in the measurement build (the shipped form when that one is not
// built).
LibbEnc libb_enc(int w, int k) {
  const Knobs& kn = knobs();
  const int la = kMeasureBuild ? kn.lib_la : kLibbEncLA;
  const int tw = kMeasureBuild ? kn.lib_wg : kLibbEncTW;
  switch (w) {
    case 3: return libb_enc_pick<3>(k, la, tw);
    case 5: return libb_enc_pick<5>(k, la, tw);
    case 7: return libb_enc_pick<7>(k, la, tw);
    case 11: return libb_enc_pick<11>(k, la, tw);
    case 13: return libb_enc_pick<13>(k, la, tw);
    default: return {nullptr, 0};
  }
}

int launch_lib(const BitApply& p, LibFn fn, uint32_t lanes, hipStream_t s) {
  const uint32_t ps = (uint32_t)(p.block_size / (uint64_t)p.w);
  const uint32_t tb = lanes * 16u;
  const uint32_t tiles = (ps + tb - 1) / tb;
  const uint64_t max_obj = (uint64_t)0x7FFFFFFF / tiles;
  for (uint64_t o0 = 0; o0 < p.nobj; o0 += max_obj) {
    const uint64_t no = (p.nobj - o0 < max_obj) ? p.nobj - o0 : max_obj;
    LibArgs a;
    a.k = p.KB;
    a.ps = ps;
    a.tiles = tiles;
    a.xmap = obj_map(tiles) ? 1u : 0u;
    uint32_t vmin = 0xFFFFFFFFu;
    for (int j = 0; j < kMaxK; ++j) {
      a.in[j] = j < p.KB ? dev_shard(p.in[j], o0) : DevShard{nullptr, 0, 0, 0};
      if (j < p.KB && a.in[j].valid < vmin) vmin = a.in[j].valid;
    }
    for (int r = 0; r < 2; ++r) {
      a.out[r] = dev_shard(p.out[r], o0);
      if (a.out[r].valid < vmin) vmin = a.out[r].valid;
    }
    a.vmin = vmin;
    hipLaunchKernelGGL(fn, dim3((uint32_t)(no * tiles)), dim3(lanes), 0, s, a);
    if (hipGetLastError() != hipSuccess) return LEOEC_E_HIP;
  }
  return LEOEC_OK;
}

}  // namespace

namespace detail {
int device_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      return 256;
    return n;
  }();
  return cus;
}
#ifdef LEOEC_MEASURE
int gfp_blocks_per_cu() { return knobs().gfp_bpc; }
#endif
// Knobs::gf8_tmap: gf8_apply workgroup -> tile order (Gf8Args::tmap), A/B only.
int gf8_tile_map() { return knobs().gf8_tmap; }
int gf8_wg_env() { return knobs().gf8_wg; }
bool gf8_tile_map_set() { return knobs().gf8_tmap_set; }
int gf8_tile_group() { return knobs().gf8_tgroup; }
}  // namespace detail

int launch(const GfApply& p, hipStream_t s) {
  if (p.K <= 0 || p.R <= 0 || (int)p.in.size() != p.K || (int)p.out.size() != p.R ||
      p.coef.size() != (size_t)p.K * p.R)
    return LEOEC_E_ARG;
  if (p.w != 8 && p.w != 16 && p.w != 32) return LEOEC_E_UNSUPPORTED;
  if (p.block_size == 0 || p.nobj == 0) return LEOEC_OK;
  if ((p.block_size & 15u) || p.block_size >= (1ull << 32)) return LEOEC_E_BAD_SIZE;
  if (!shards_ok(p.in) || !shards_ok(p.out)) return LEOEC_E_ARG;
  const uint32_t tiles = (uint32_t)((p.block_size + kTileBytes - 1) / kTileBytes);
  // objects per launch bounded for the narrowest tiles (1 KiB, gf8_apply's
  // 64-lane form) so no grid exceeds 2^31 - 1 workgroups
  const uint64_t max_obj = (uint64_t)0x7FFFFFFF / ((p.block_size + 1023) / 1024);
  for (uint64_t o0 = 0; o0 < p.nobj; o0 += max_obj) {
    const uint64_t no = (p.nobj - o0 < max_obj) ? p.nobj - o0 : max_obj;
    for (int r0 = 0; r0 < p.R; r0 += kMaxR) {
      const int nr = (p.R - r0 < kMaxR) ? p.R - r0 : kMaxR;
      // inputs beyond 16 are folded in by accumulating launches (ACC)
      for (int j0 = 0; j0 < p.K; j0 += kMaxK) {
        const int nk = (p.K - j0 < kMaxK) ? p.K - j0 : kMaxK;
        const Chunk c{r0, nr, j0, nk, o0, no, tiles};
        ChunkFn fn;
        if (p.w == 8) {
          fn = gf8_pick(std::make_index_sequence<kMaxK>{}, nk, nr, j0 > 0);
#ifdef LEOEC_MEASURE
          if (nk == 10 && nr == 4 && j0 == 0) {
            const int var = knobs().gf8_variant;
            if (var > 0 && gf8_variant(var)) fn = gf8_variant(var);
          }
#endif
        } else {
          const Knobs& kn = knobs();
          const int form = kMeasureBuild ? kn.gfw_form : 3;
          if (form == 3)
            fn = gfs_pick(p.w, nr, j0 > 0);
#ifdef LEOEC_MEASURE
          else if (form == 0)
            fn = p.w == 16 ? gfp_pick<16>(nr, j0 > 0, kn.gfp_cpt)
                           : gfp_pick<32>(nr, j0 > 0, kn.gfp_cpt);
          else if (form == 1 && p.w == 16)
            fn = gf16_pick(nr, j0 > 0);
          else
            fn = p.w == 16 ? gfw_pick<16>(nr, j0 > 0) : gfw_pick<32>(nr, j0 > 0);
#else
          else
            return LEOEC_E_UNSUPPORTED;
#endif
        }
        const int rc = fn(p, c, s);
        if (rc) return rc;
      }
    }
  }
  return LEOEC_OK;
}

namespace {
using LibDecFn = void (*)(const detail::LibDecArgs);
// Knobs::lib_dec_wg = 64 (measurement build): 64-lane workgroups, 1 KiB tiles.
uint32_t lib_dec_lanes() { return kMeasureBuild && knobs().lib_dec_wg == 64 ? 64u : (uint32_t)kThreads; }
LibbDec libb_dec(int w, int k) {
  const Knobs& kn = knobs();
  const int la = kMeasureBuild && kn.lib_dec_la >= 0 ? kn.lib_dec_la : libb_dec_la(w, k);
  const int tw = kMeasureBuild && kn.lib_dec_wg > 0 ? kn.lib_dec_wg : kLibbDecTW;
  switch (w) {
    case 3: return libb_dec_pick<3>(k, la, tw);
    case 5: return libb_dec_pick<5>(k, la, tw);
    case 7: return libb_dec_pick<7>(k, la, tw);
    case 11: return libb_dec_pick<11>(k, la, tw);
    case 13: return libb_dec_pick<13>(k, la, tw);
    default: return {nullptr, 0};
  }
}
// (the round-1 syndrome kernel: measurement build only since round 5)
template <int W>
LibDecFn lib_dec_kernel_w() {
#ifdef LEOEC_MEASURE
  if (lib_dec_lanes() == 64) return &detail::lib_dec_apply<W, 64>;
  return &detail::lib_dec_apply<W>;
#else
  return nullptr;
#endif
}
LibDecFn lib_dec_kernel(int w) {
  switch (w) {
    case 3: return lib_dec_kernel_w<3>();
    case 5: return lib_dec_kernel_w<5>();
    case 7: return lib_dec_kernel_w<7>();
    case 11: return lib_dec_kernel_w<11>();
    case 13: return lib_dec_kernel_w<13>();
    default: return nullptr;
  }
}
}  // namespace

bool lib_dec_supported(int w) {
  return knobs().lib_form != 0 && (w == 3 || w == 5 || w == 7 || w == 11 || w == 13);
}

int launch(const LibDecApply& p, hipStream_t s) {
  const int w = p.w;
  LibDecFn fn = nullptr;
  uint32_t lanes = 0;
  if (knobs().lib_buf != 0) {  // shipped: libb_dec_apply
    const LibbDec b = libb_dec(w, p.k);
    fn = b.fn;
    lanes = b.lanes;
  }
  if (!fn) {
    fn = lib_dec_kernel(w);
    lanes = lib_dec_lanes();
  }
  const int nout = (int)p.out.size();
  if (!fn || p.k <= 0 || p.k > w || (int)p.data.size() != p.k || p.cod.size() != 2 || nout < 1 ||
      nout > 2 || p.mbits.size() != (size_t)nout * 2 * w)
    return LEOEC_E_ARG;
  if (p.block_size == 0 || p.nobj == 0) return LEOEC_OK;
  if (p.block_size % ((uint64_t)16 * w) || p.block_size >= (1ull << 32)) return LEOEC_E_BAD_SIZE;
  for (const auto* v : {&p.data, &p.cod, &p.out})
    for (const Shard& sh : *v)
      if (sh.base && (((uintptr_t)sh.base & 15u) || (sh.stride & 15u))) return LEOEC_E_ARG;
  const uint32_t ps = (uint32_t)(p.block_size / (uint64_t)w);
  const uint32_t tb = lanes * 16u;
  const uint32_t tiles = (ps + tb - 1) / tb;
  const uint64_t max_obj = (uint64_t)0x7FFFFFFF / tiles;
  for (uint64_t o0 = 0; o0 < p.nobj; o0 += max_obj) {
    const uint64_t no = (p.nobj - o0 < max_obj) ? p.nobj - o0 : max_obj;
    LibDecArgs a;
    a.k = p.k;
    a.nout = nout;
    a.ps = ps;
    a.tiles = tiles;
    a.xmap = obj_map(tiles) ? 1u : 0u;
    uint32_t vmin = 0xFFFFFFFFu;
    auto take = [&](const Shard& sh) {
      if (!sh.base) return DevShard{nullptr, 0, 0, 0};
      const DevShard d = dev_shard(sh, o0);
      if (d.valid < vmin) vmin = d.valid;
      return d;
    };
    for (int j = 0; j < kMaxK; ++j) a.data[j] = j < p.k ? take(p.data[j]) : DevShard{nullptr, 0, 0, 0};
    for (int r = 0; r < 2; ++r) a.cod[r] = take(p.cod[r]);
    for (int b = 0; b < 2; ++b) {
      a.out[b] = b < nout ? take(p.out[b]) : DevShard{nullptr, 0, 0, 0};
      for (int q = 0; q < 32; ++q)
        a.mbits[b][q] = (b < nout && q < 2 * w) ? p.mbits[(size_t)b * 2 * w + q] : 0u;
    }
    a.vmin = vmin;
    hipLaunchKernelGGL(fn, dim3((uint32_t)(no * tiles)), dim3(lanes), 0, s, a);
    if (hipGetLastError() != hipSuccess) return LEOEC_E_HIP;
  }
  return LEOEC_OK;
}

int launch(const BitApply& p, hipStream_t s) {
  const int w = p.w;
  if (w <= 0 || w > 32 || p.KB <= 0 || p.RB <= 0 || (int)p.in.size() != p.KB ||
      (int)p.out.size() != p.RB || p.bits.size() != (size_t)p.RB * w * p.KB * w)
    return LEOEC_E_ARG;
  if (p.block_size == 0 || p.nobj == 0) return LEOEC_OK;
  if (p.block_size % ((uint64_t)16 * w) || p.block_size >= (1ull << 32)) return LEOEC_E_BAD_SIZE;
  if (!shards_ok(p.in) || !shards_ok(p.out)) return LEOEC_E_ARG;
  if (knobs().lib_form != 0 && is_liberation_encode(p)) {
    const int buf = knobs().lib_buf;
    if (buf > 0 || (buf < 0 && w >= kLibbEncMinW)) {
      const LibbEnc b = libb_enc(w, p.KB);
      if (b.fn) return launch_lib(p, b.fn, b.lanes, s);
    }
    if (const LibFn lf = lib_kernel(w)) return launch_lib(p, lf, lib_lanes(), s);
  }
  const uint32_t ps = (uint32_t)(p.block_size / (uint64_t)w);
  const uint32_t tiles = (ps + kTileBytes - 1) / kTileBytes;
  const uint64_t max_obj = (uint64_t)0x7FFFFFFF / tiles;
  const int blocks_per_pass = kMaxPk / w;  // output blocks whose packets fit one launch
  const int KPtot = p.KB * w;
  for (uint64_t o0 = 0; o0 < p.nobj; o0 += max_obj) {
    const uint64_t no = (p.nobj - o0 < max_obj) ? p.nobj - o0 : max_obj;
    for (int b0 = 0; b0 < p.RB; b0 += blocks_per_pass) {
      const int nb = (p.RB - b0 < blocks_per_pass) ? p.RB - b0 : blocks_per_pass;
      const int RP = nb * w;
      for (int j0 = 0; j0 < p.KB; j0 += kMaxK) {
        const int nk = (p.KB - j0 < kMaxK) ? p.KB - j0 : kMaxK;
        BitArgs a;
        a.w = w;
        a.KP = nk * w;
        a.ps = ps;
        a.tiles = tiles;
        for (int j = 0; j < kMaxK; ++j)
          a.in[j] = j < nk ? dev_shard(p.in[j0 + j], o0) : DevShard{nullptr, 0, 0, 0};
        for (int o = 0; o < kMaxPk; ++o) {
          a.out[o] = DevShard{nullptr, 0, 0, 0};
          if (o >= RP) continue;
          const Shard& sh = p.out[b0 + o / w];
          const uint64_t pk = (uint64_t)(o % w) * ps;
          DevShard d = dev_shard(sh, o0);
          d.base += pk;
          const uint64_t v = sh.valid > pk ? sh.valid - pk : 0;
          d.valid = (uint32_t)(v < ps ? v : ps);
          a.out[o] = d;
        }
        for (int q = 0; q < kMaxK * 32; ++q) {
          uint32_t word = 0;
          if (q < nk * w)
            for (int o = 0; o < RP; ++o)
              if (p.bits[(size_t)(b0 * w + o) * KPtot + (size_t)j0 * w + q]) word |= 1u << (31 - o);
          a.bits[q] = word;
        }
        const bool acc = j0 > 0;
        const dim3 grid((uint32_t)(no * tiles)), block(kThreads);
        BitFn fn = bit_kernel_even(std::make_index_sequence<16>{}, RP, acc);
#ifdef LEOEC_MEASURE
        // bit_form 8: the shipped form at the {8,16,32} sizes (A/B)
        const int form = knobs().bit_form;
        const int ro = RP <= 8 ? 8 : RP <= 16 ? 16 : 32;
        if (form != 4) fn = bit_kernel(ro, acc, form == 8 ? 4 : form);
#endif
        hipLaunchKernelGGL(fn, grid, block, 0, s, a);
        if (hipGetLastError() != hipSuccess) return LEOEC_E_HIP;
      }
    }
  }
  return LEOEC_OK;
}

}  // namespace leoec
