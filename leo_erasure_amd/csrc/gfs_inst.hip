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

namespace leoec {
namespace detail {

template <int R>
struct GfsArgs {
  DevShard in[kMaxK];
  DevShard out[R];
  uint32_t coef[R][kMaxK];
  int K;
  uint32_t tiles;  // tiles per object
  uint32_t vmin;   // min valid over all shards of the launch
  uint32_t xmap;   // 1: xcd_obj_map (objects of <= kObjMapMaxTiles tiles)
};

constexpr int kGfsLanes = 64;

constexpr int kGfsRegs = 16;  // registers per value (64 bytes per lane)
constexpr int kGfsLoads = kGfsRegs / 4;
constexpr uint32_t kGfsTile = kGfsLanes * 16u * kGfsLoads;

__device__ __forceinline__ void gfs_load(const DevShard& s, uint64_t o, uint32_t t0, bool full,
                                         uint32_t (&rows)[kGfsRegs]) {
  constexpr int NL = kGfsLoads;
  const uint8_t* p = s.base + o * s.stride;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint32_t off = t0 + (uint32_t)i * (kGfsLanes * 16u) + threadIdx.x * 16u;
    const u32x4 v = full ? ld16<true>(p + off) : load_guarded(p, off, s.valid);
#pragma unroll
    for (int e = 0; e < 4; ++e) rows[4 * i + e] = v[e];
  }
}

// Input j (raw words in pl) into the R accumulators.
template <int W, int R>
__device__ __forceinline__ void gfs_step(const GfsArgs<R>& a, int j, uint32_t (&pl)[kGfsRegs],
                                         uint32_t (&acc)[R][kGfsRegs]) {
  gfs::transpose<kGfsRegs>(pl);
  uint32_t c[R];
#pragma unroll
  for (int r = 0; r < R; ++r) c[r] = a.coef[r][j];
  if constexpr (W == 32) gfs::mac_p32<R>(pl, acc, c);
  else gfs::mac<16, R>(pl, acc, c);
}

template <int W, int R, bool ACC>
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
      gfs_load(a.out[r], o, t0, full, acc[r]);
      gfs::transpose<kGfsRegs>(acc[r]);
    } else {
#pragma unroll
      for (int k = 0; k < kGfsRegs; ++k) acc[r][k] = 0u;
    }
  }
  // two input buffers: input j+1 is loaded into one while input j is
  // transposed and accumulated in place in the other
  const int K = a.K;
  uint32_t bufa[kGfsRegs], bufb[kGfsRegs];
  gfs_load(a.in[0], o, t0, full, bufa);
  for (int j = 0; j < K; j += 2) {
    if (j + 1 < K) gfs_load(a.in[j + 1], o, t0, full, bufb);
    gfs_step<W, R>(a, j, bufa, acc);
    if (j + 1 >= K) break;
    if (j + 2 < K) gfs_load(a.in[j + 2], o, t0, full, bufa);
    gfs_step<W, R>(a, j + 1, bufb, acc);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    gfs::transpose<kGfsRegs>(acc[r]);
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

template <int W, int R, bool ACC>
int launch_gfs_t(const GfApply& p, const Chunk& c, hipStream_t s) {
  GfsArgs<R> a;
  uint32_t vmin = 0xFFFFFFFFu;
  a.K = c.nk;
  for (int j = 0; j < kMaxK; ++j) {
    a.in[j] = j < c.nk ? dev_shard(p.in[c.j0 + j], c.o0) : DevShard{nullptr, 0, 0, 0};
    if (j < c.nk) vmin = a.in[j].valid < vmin ? a.in[j].valid : vmin;
  }
  for (int r = 0; r < R; ++r) {
    a.out[r] = dev_shard(p.out[c.r0 + r], c.o0);
    vmin = a.out[r].valid < vmin ? a.out[r].valid : vmin;
    for (int j = 0; j < kMaxK; ++j)
      a.coef[r][j] = j < c.nk ? p.coef[(size_t)(c.r0 + r) * p.K + c.j0 + j] : 0u;
  }
  a.tiles = (uint32_t)((p.block_size + kGfsTile - 1) / kGfsTile);
  a.vmin = vmin;
  a.xmap = a.tiles <= kObjMapMaxTiles ? 1u : 0u;
  const uint64_t grid = c.no * a.tiles;
  if (grid == 0 || grid > 0x7FFFFFFFull) return LEOEC_E_ARG;
  hipLaunchKernelGGL((gfs_apply<W, R, ACC>), dim3((uint32_t)grid), dim3(kGfsLanes), 0, s, a);
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
  return w == 16 ? gfs_pick_w<16>(r, acc) : gfs_pick_w<32>(r, acc);
}

}  // namespace detail
}  // namespace leoec
