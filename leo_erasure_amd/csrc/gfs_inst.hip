// gfs_inst.hip — bitsliced GF(2^16) / GF(2^32) kernel (gfs_apply) and its
// launches: vandrs w = 16 / 32 encode, decode and repair
// (jerasure_matrix_encode / _decode_data / _decode_selected over words,
// c_src/rscoding.cpp:71,147,198).  The arithmetic is gfs_core.hpp.
//
// One 64-lane workgroup per tile: each lane loads 64 bytes of every input
// block (4 global_load_dwordx4, a wave reading 1 KiB contiguous per load) —
// 32 words at w = 16, 16 words at w = 32 — transposes them into bit-planes
// (16 registers either way: gfs_core.hpp, the w = 32 "packed" layout) and
// accumulates c_rj * x_j for its R output rows in the plane domain; the next
// input's loads are issued before the current input's arithmetic.  The R
// accumulators are transposed back and stored once.  A tile is 4 KiB per
// block.  16 registers per value keep a 4-row w = 32 launch at ~110 VGPRs
// (4 waves per SIMD); the 32-words-per-lane form needed 229 (2 waves) and
// ran ~15 % slower.
#include "gfs_core.hpp"
#include "kernels_impl.hpp"
#include "knobs.hpp"

namespace leoec {
namespace detail {

template <int R>
struct GfsArgs {
  InCol col[kMaxK + 1];  // col[K]: empty (valid 0), the target of the last prefetch
  InCol ones;            // a column of 0/1 coefficients done in the word domain (or empty)
  DevShard out[R];
  int K;                  // bitsliced columns, >= 1
  uint32_t tiles;  // tiles per object
  uint32_t vmin;   // min valid over all shards of the launch
  uint32_t xmap;   // 1: xcd_obj_map (objects of <= kObjMapMaxTiles tiles)
};

constexpr int kGfsLanes = 64;

constexpr int kGfsRegs = 16;  // registers per value (64 bytes per lane)
constexpr int kGfsLoads = kGfsRegs / 4;
constexpr uint32_t kGfsTile = kGfsLanes * 16u * kGfsLoads;

// Loads go through shard_rsrc() (16-byte chunks): every load is
// unconditional and the bytes of the one chunk that straddles `valid` are
// cleared by gfs_tail() in tiles that are not full.  An input index >= K gets
// an empty range (col[K], valid 0): the loop's prefetch of "input K" returns
// zeros.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gfs_rsrc(const uint8_t* base, uint64_t stride,
                                                           uint32_t valid, uint64_t o) {
  return shard_rsrc(base, stride, valid, o, 16u);
}

__device__ __forceinline__ void gfs_load(__amdgpu_buffer_rsrc_t rs, uint32_t t0,
                                         uint32_t (&rows)[kGfsRegs]) {
#pragma unroll
  for (int i = 0; i < kGfsLoads; ++i) {
    const uint32_t off = t0 + (uint32_t)i * (kGfsLanes * 16u) + threadIdx.x * 16u;
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2);
#pragma unroll
    for (int e = 0; e < 4; ++e) rows[4 * i + e] = v[e];
  }
}

// Clear the bytes at or past `valid` (tiles that are not full only).
__device__ __forceinline__ void gfs_tail(uint32_t t0, uint32_t valid, uint32_t (&rows)[kGfsRegs]) {
#pragma unroll
  for (int i = 0; i < kGfsLoads; ++i) {
    const uint32_t off = t0 + (uint32_t)i * (kGfsLanes * 16u) + threadIdx.x * 16u;
    const uint32_t n = off >= valid ? 0u : (valid - off > 16u ? 16u : valid - off);
    const u32x4 v = keep_first(u32x4{rows[4 * i], rows[4 * i + 1], rows[4 * i + 2], rows[4 * i + 3]}, n);
#pragma unroll
    for (int e = 0; e < 4; ++e) rows[4 * i + e] = v[e];
  }
}

// Input j (raw words in pl) into the R accumulators.  MODE (measurement
// builds only; not a code): 1 every coefficient forced to 0xFFFFFFFF at run
// time (an opaque scalar the compiler cannot fold: the shipped tests and
// branches run, all taken), 2 the same VALU work with no tests compiled in
// (gfs_core.hpp ALLB).
template <int W, int R, int MODE = 0>
__device__ __forceinline__ void gfs_step(const InCol& col, uint32_t t0, bool full,
                                         uint32_t (&pl)[kGfsRegs], uint32_t (&acc)[R][kGfsRegs]) {
  if (!full) gfs_tail(t0, col.valid, pl);
  gfs::transpose<kGfsRegs>(pl);
  uint32_t c[R];
  uint32_t force = 0u;
  if constexpr (MODE == 1) asm volatile("s_mov_b32 %0, -1" : "=s"(force));  // opaque: tests stay
#pragma unroll
  for (int r = 0; r < R; ++r) c[r] = col.coef[r] | force;
  if constexpr (W == 32) gfs::mac_p32<R, MODE == 2>(pl, acc, c);
  else gfs::mac<16, R>(pl, acc, c);
}

// PF (measurement builds): inputs whose loads are in flight while one is
// computed (1 shipped: two input buffers; 2: three).
template <int W, int R, bool ACC, int MODE = 0, int PF = 1>
__global__ void __launch_bounds__(kGfsLanes) __attribute__((amdgpu_waves_per_eu(4)))
gfs_apply(const GfsArgs<R> a) {
  constexpr int NL = kGfsLoads;
  constexpr uint32_t TB = kGfsTile;
  const uint32_t b = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = b / a.tiles;
  const uint32_t t0 = (b - obj * a.tiles) * TB;
  const bool full = t0 + TB <= a.vmin;  // wave-uniform
  const uint64_t o = obj;
  uint32_t acc[R][kGfsRegs];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (ACC) {
      gfs_load(gfs_rsrc(a.out[r].base, a.out[r].stride, a.out[r].valid, o), t0, acc[r]);
      if (!full) gfs_tail(t0, a.out[r].valid, acc[r]);
      gfs::transpose<kGfsRegs>(acc[r]);
    } else {
#pragma unroll
      for (int k = 0; k < kGfsRegs; ++k) acc[r][k] = 0u;
    }
  }
  // two input buffers: input j+1 is loaded into one while input j is
  // transposed and accumulated in place in the other
  const int K = a.K;
  if constexpr (PF == 2) {
    // three input buffers: inputs j+1 and j+2 in flight while j is computed
    uint32_t b0[kGfsRegs], b1[kGfsRegs], b2[kGfsRegs];
    auto col = [&](int i) { return a.col[i < K ? i : K]; };
    InCol c0 = col(0), c1 = col(1), c2 = col(2);
    gfs_load(gfs_rsrc(c0.base, c0.stride, c0.valid, o), t0, b0);
    gfs_load(gfs_rsrc(c1.base, c1.stride, c1.valid, o), t0, b1);
    for (int j = 0;; j += 3) {
      gfs_load(gfs_rsrc(c2.base, c2.stride, c2.valid, o), t0, b2);
      const InCol c3 = col(j + 3);
      gfs_step<W, R, MODE>(c0, t0, full, b0, acc);
      if (j + 1 >= K) break;
      gfs_load(gfs_rsrc(c3.base, c3.stride, c3.valid, o), t0, b0);
      const InCol c4 = col(j + 4);
      gfs_step<W, R, MODE>(c1, t0, full, b1, acc);
      if (j + 2 >= K) break;
      gfs_load(gfs_rsrc(c4.base, c4.stride, c4.valid, o), t0, b1);
      const InCol c5 = col(j + 5);
      gfs_step<W, R, MODE>(c2, t0, full, b2, acc);
      if (j + 3 >= K) break;
      c0 = c3;
      c1 = c4;
      c2 = c5;
    }
  } else {
  uint32_t bufa[kGfsRegs], bufb[kGfsRegs];
  InCol cur = a.col[0], nx = a.col[K > 1 ? 1 : K];
  gfs_load(gfs_rsrc(cur.base, cur.stride, cur.valid, o), t0, bufa);
  for (int j = 0;; j += 2) {
    gfs_load(gfs_rsrc(nx.base, nx.stride, nx.valid, o), t0, bufb);  // input j+1 (or empty)
    const InCol nx2 = a.col[j + 2 < K ? j + 2 : K];
    gfs_step<W, R, MODE>(cur, t0, full, bufa, acc);
    if (j + 1 >= K) break;
    gfs_load(gfs_rsrc(nx2.base, nx2.stride, nx2.valid, o), t0, bufa);  // input j+2 (or empty)
    const InCol nx3 = a.col[j + 3 < K ? j + 3 : K];
    gfs_step<W, R, MODE>(nx, t0, full, bufb, acc);
    if (j + 2 >= K) break;
    cur = nx2;
    nx = nx3;
  }
  }
  // A column of zeros and ones (encode's column 0) skips the bit domain: it
  // is XORed into the accumulators after these are transposed back to
  // words, which saves its transpose and every doubling step.  Its load is
  // in flight during the transposes; an empty `ones` (no such column) reads
  // zeros and has no coefficient set.
  const InCol oc = a.ones;
  uint32_t bufc[kGfsRegs];  // (loading into bufa here put the loop's loads in waterfall loops)
  gfs_load(gfs_rsrc(oc.base, oc.stride, oc.valid, o), t0, bufc);
#pragma unroll
  for (int r = 0; r < R; ++r) gfs::transpose<kGfsRegs>(acc[r]);
  if (!full) gfs_tail(t0, oc.valid, bufc);
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (oc.coef[r] & 1u) {
#pragma unroll
      for (int i = 0; i < kGfsRegs; ++i) acc[r][i] ^= bufc[i];
    }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    uint8_t* p = const_cast<uint8_t*>(a.out[r].base) + o * a.out[r].stride;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const uint32_t off = t0 + (uint32_t)i * (kGfsLanes * 16u) + threadIdx.x * 16u;
      const u32x4 v = {acc[r][4 * i], acc[r][4 * i + 1], acc[r][4 * i + 2], acc[r][4 * i + 3]};
      if (full) st16<true>(p + off, v);
      else store_guarded(p, off, a.out[r].valid, v);
    }
  }
}

template <int W, int R, bool ACC, int MODE = 0, int PF = 1>
int launch_gfs_t(const GfApply& p, const Chunk& c, hipStream_t s) {
  GfsArgs<R> a;
  uint32_t vmin = 0xFFFFFFFFu;
  // at most one column whose coefficients are all 0 or 1 goes to `ones`, if
  // another column remains bitsliced
  int order[kMaxK], n = 0, ones = -1;
  for (int j = 0; j < c.nk; ++j) {
    bool is01 = ones < 0 && c.nk > 1;
    for (int r = 0; r < R; ++r) is01 = is01 && p.coef[(size_t)(c.r0 + r) * p.K + c.j0 + j] <= 1u;
    if (is01) ones = j;
    else order[n++] = j;
  }
  a.K = n;
  auto fill = [&](InCol& col, int j) {
    col = InCol{};
    const DevShard d = dev_shard(p.in[c.j0 + j], c.o0);
    col.base = d.base;
    col.stride = d.stride;
    col.valid = d.valid;
    vmin = d.valid < vmin ? d.valid : vmin;
    for (int r = 0; r < R; ++r) col.coef[r] = p.coef[(size_t)(c.r0 + r) * p.K + c.j0 + j];
  };
  for (int x = 0; x <= kMaxK; ++x) {
    if (x < n) {
      fill(a.col[x], order[x]);
    } else {
      a.col[x] = InCol{};
      a.col[x].base = a.col[0].base;  // empty range: never dereferenced
    }
  }
  if (ones >= 0) {
    fill(a.ones, ones);
  } else {
    a.ones = InCol{};
    a.ones.base = a.col[0].base;
  }
  for (int r = 0; r < R; ++r) {
    a.out[r] = dev_shard(p.out[c.r0 + r], c.o0);
    vmin = a.out[r].valid < vmin ? a.out[r].valid : vmin;
  }
  a.tiles = (uint32_t)((p.block_size + kGfsTile - 1) / kGfsTile);
  a.vmin = vmin;
  a.xmap = a.tiles <= kObjMapMaxTiles ? 1u : 0u;
  const uint64_t grid = c.no * a.tiles;
  if (grid == 0 || grid > 0x7FFFFFFFull) return LEOEC_E_ARG;
  hipLaunchKernelGGL((gfs_apply<W, R, ACC, MODE, PF>), dim3((uint32_t)grid), dim3(kGfsLanes), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

template <int W>
ChunkFn gfs_pick_w(int r, bool acc) {
  static const ChunkFn tbl[2][kMaxR] = {
      {&launch_gfs_t<W, 1, false>, &launch_gfs_t<W, 2, false>, &launch_gfs_t<W, 3, false>,
       &launch_gfs_t<W, 4, false>},
      {&launch_gfs_t<W, 1, true>, &launch_gfs_t<W, 2, true>, &launch_gfs_t<W, 3, true>,
       &launch_gfs_t<W, 4, true>}};
  return tbl[acc ? 1 : 0][r - 1];
}

ChunkFn gfs_pick(int w, int r, bool acc) {
#ifdef LEOEC_MEASURE
  // LEOEC_GFS_MODE=1|2 (w = 32, 4 rows, one input chunk; timing only, wrong bytes)
  const int mode = knobs().gfs_mode;
  if (w == 32 && r == 4 && !acc && mode == 1) return &launch_gfs_t<32, 4, false, 1>;
  if (w == 32 && r == 4 && !acc && mode == 2) return &launch_gfs_t<32, 4, false, 2>;
  // LEOEC_GFS_PF=2: two inputs in flight (4 rows, one input chunk)
  if (r == 4 && !acc && knobs().gfs_pf == 2)
    return w == 16 ? &launch_gfs_t<16, 4, false, 0, 2> : &launch_gfs_t<32, 4, false, 0, 2>;
#endif
  return w == 16 ? gfs_pick_w<16>(r, acc) : gfs_pick_w<32>(r, acc);
}

}  // namespace detail
}  // namespace leoec
