// cbm_inst.hip — cauchyrs(10,4,8) encode with its bitmatrix compiled in
// (BASELINE configs[3]: the reference runs it as jerasure_schedule_encode
// over packets of blockSize / w bytes, c_src/cauchycoding.cpp:38-40,72).
//
// The encode bitmatrix of cauchy_good_general_coding_matrix(10, 4, 8) is a
// constant: 32 output packets x 80 input packets, 888 ones.  With it known
// at compile time the encode is a pure XOR schedule: every input packet is
// loaded once (16 bytes per lane, one raw buffer load), XORed straight into
// the output packets its bitmatrix column names — static register indices,
// no doubling chain, no masks, no coefficient branches — and dropped, so a
// lane holds only the 32 output packets (128 VGPRs) plus the loads in
// flight, at the 16-byte lane width the access pattern prefers
// (profiles/r02_v15_packet_ceiling_*.log).  The matrix is recomputed here by
// the same construction as codes.cpp cauchy_good_coding_matrix (cauchy
// original 1/(i ^ (m + j)), columns scaled to a row of ones, each later row
// divided by its weight-minimising element) in constexpr code, and the
// launcher takes this kernel only when the plan's coefficient rows equal it
// (launch_cbm), so a mismatch can only route a call to the generic kernel.
//
// Measured against the shipped bitsliced kernel (gfbit_apply, 8-byte lanes)
// in one process (profiles/r03_v9_ab_cauchy_compiled_bitmatrix*.log): 0.715
// against 0.712 at 1,024 objects, 0.680 against 0.718 at 4,096 — the access
// pattern of 13,120-byte packets, not the arithmetic, sets the rate — so it
// is a measurement-build form (LEOEC_GFBIT_CBM); the product library
// compiles only the stub below.
#include <utility>

#include "kernels_impl.hpp"
#include "knobs.hpp"

namespace leoec {
namespace detail {

#ifndef LEOEC_MEASURE
bool launch_cbm(const GfBitApply&, hipStream_t, int*) { return false; }
#else

// ---- constexpr GF(2^8), polynomial 0x11D (gf-complete's default) ----------
constexpr uint32_t cgf_mul(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) {
    if (b & 1u) r ^= a;
    b >>= 1;
    a <<= 1;
    if (a & 0x100u) a ^= 0x11Du;
  }
  return r;
}
constexpr uint32_t cgf_inv(uint32_t a) {
  for (uint32_t x = 1; x < 256; ++x)
    if (cgf_mul(a, x) == 1u) return x;
  return 0;
}
constexpr int cgf_popcount(uint32_t v) {
  int n = 0;
  for (; v; v &= v - 1) ++n;
  return n;
}
constexpr int cgf_weight(uint32_t c) {  // ones of c's 8 x 8 bitmatrix
  int n = 0;
  for (int x = 0; x < 8; ++x) n += cgf_popcount(cgf_mul(c, 1u << x));
  return n;
}

// cauchy_good_general_coding_matrix(K, M, 8) for M > 2 and its bitmatrix.
template <int K, int M>
struct CauchyGood8 {
  static_assert(M > 2 && K + M <= 256, "the cauchy_original + improve path");
  uint32_t c[M][K] = {};
  bool b[M * 8][K * 8] = {};  // b[i*8 + l][j*8 + x] = bit l of c[i][j] * 2^x
  int ones = 0;
  constexpr CauchyGood8() {
    for (int i = 0; i < M; ++i)
      for (int j = 0; j < K; ++j) c[i][j] = cgf_inv((uint32_t)(i ^ (M + j)));
    for (int j = 0; j < K; ++j) {
      if (c[0][j] == 1u) continue;
      const uint32_t s = cgf_inv(c[0][j]);
      for (int i = 0; i < M; ++i) c[i][j] = cgf_mul(c[i][j], s);
    }
    for (int i = 1; i < M; ++i) {
      int best = 0;
      for (int j = 0; j < K; ++j) best += cgf_weight(c[i][j]);
      int pick = -1;
      for (int j = 0; j < K; ++j) {
        if (c[i][j] == 1u) continue;
        const uint32_t s = cgf_inv(c[i][j]);
        int wt = 0;
        for (int x = 0; x < K; ++x) wt += cgf_weight(cgf_mul(c[i][x], s));
        if (wt < best) {
          best = wt;
          pick = j;
        }
      }
      if (pick >= 0) {
        const uint32_t s = cgf_inv(c[i][pick]);
        for (int j = 0; j < K; ++j) c[i][j] = cgf_mul(c[i][j], s);
      }
    }
    for (int i = 0; i < M; ++i)
      for (int j = 0; j < K; ++j)
        for (int x = 0; x < 8; ++x) {
          const uint32_t v = cgf_mul(c[i][j], 1u << x);
          for (int l = 0; l < 8; ++l) {
            b[i * 8 + l][j * 8 + x] = (v >> l) & 1u;
            ones += (v >> l) & 1u;
          }
        }
  }
};

struct Cbm10_4 {
  static constexpr int K = 10, M = 4;
  static constexpr CauchyGood8<10, 4> m{};
};
// cauchy_good(10,4,8) has 888 bitmatrix ones, row 0
// all ones, row 1 = 97 ac 1 e1 a6 9e 2c d e2 36.
static_assert(Cbm10_4::m.ones == 888, "cauchy_good(10,4,8) bitmatrix weight");
static_assert(Cbm10_4::m.c[0][3] == 1u && Cbm10_4::m.c[1][0] == 0x97u &&
                  Cbm10_4::m.c[1][1] == 0xACu && Cbm10_4::m.c[3][9] == 0x22u,
              "cauchy_good(10,4,8) coefficients");

struct CbmArgs {
  DevShard in[kMaxK];
  DevShard out[kMaxR];
  uint32_t ps;     // packet bytes (bs / 8)
  uint32_t bs;     // block bytes
  uint32_t tiles;  // tiles per object (over one packet)
  uint32_t xmap;   // 1: xcd_obj_map
};

// Input packet P = (block P / 8, packet P % 8): load it, XOR it into every
// output packet O with b[O][P] set (a constant: the fold keeps only those).
// Pins an accumulator's value in its registers at this point: without it
// the compiler sinks the XORs toward the final stores and keeps the input
// packets alive instead (all 80: 320 VGPRs, spilled).
__device__ __forceinline__ void cbm_pin(u32x4& x) { asm volatile("" : "+v"(x)); }

template <class BM, int P, int... O>
__device__ __forceinline__ void cbm_column(u32x4 (&acc)[BM::M * 8], const u32x4& v,
                                           std::integer_sequence<int, O...>) {
  ((BM::m.b[O][P] ? (void)(acc[O] ^= v, cbm_pin(acc[O])) : (void)0), ...);
}

// Packet P's load into its ring slot (P past the last packet: nothing).
template <class BM, int D, int P>
__device__ __forceinline__ void cbm_load(u32x4 (&ring)[D + 1],
                                         const __amdgpu_buffer_rsrc_t (&rs)[BM::K], uint32_t ps,
                                         uint32_t off) {
  if constexpr (P < BM::K * 8) {
    constexpr int J = P / 8, X = P % 8;
    // lane offset in a VGPR, packet offset in an SGPR (one VGPR for all 8)
    ring[P % (D + 1)] = __builtin_amdgcn_raw_buffer_load_b128(
        rs[J], off, __builtin_amdgcn_readfirstlane((uint32_t)X * ps), 2);  // nt; past `valid`: 0
  }
}

// Step P: issue packet P + D's load, then XOR packet P (loaded D steps ago)
// into its output packets.  The scheduling barrier keeps each load at its
// step: left free, the scheduler hoists all 80 loads (320 VGPRs) and spills.
template <class BM, int D, int P>
__device__ __forceinline__ void cbm_step(u32x4 (&acc)[BM::M * 8], u32x4 (&ring)[D + 1],
                                         const __amdgpu_buffer_rsrc_t (&rs)[BM::K],
                                         const uint32_t (&valid)[BM::K], uint32_t ps, uint32_t bs,
                                         uint32_t off) {
  constexpr int J = P / 8, X = P % 8;
  cbm_load<BM, D, P + D>(ring, rs, ps, off);
  u32x4 v = ring[P % (D + 1)];
  const uint32_t at = (uint32_t)X * ps + off;
  if (valid[J] < bs) v = keep_first(v, valid[J] > at ? valid[J] - at : 0u);  // wave-uniform test
  cbm_column<BM, P>(acc, v, std::make_integer_sequence<int, BM::M * 8>{});
  __builtin_amdgcn_sched_barrier(0);
}

template <class BM, int D, int... P>
__device__ __forceinline__ void cbm_all(u32x4 (&acc)[BM::M * 8],
                                        const __amdgpu_buffer_rsrc_t (&rs)[BM::K],
                                        const uint32_t (&valid)[BM::K], uint32_t ps, uint32_t bs,
                                        uint32_t off, std::integer_sequence<int, P...>) {
  u32x4 ring[D + 1];
  ((P < D ? cbm_load<BM, D, P>(ring, rs, ps, off) : (void)0), ...);  // the first D packets
  __builtin_amdgcn_sched_barrier(0);
  (cbm_step<BM, D, P>(acc, ring, rs, valid, ps, bs, off), ...);
}

// D: input packets in flight (a ring of D + 1 packet registers).
template <class BM, int TW, int WAVES, int D>
__global__ void __launch_bounds__(TW) __attribute__((amdgpu_waves_per_eu(WAVES, 8)))
cbm_apply(const CbmArgs a) {
  constexpr int K = BM::K, NO = BM::M * 8;
  const uint32_t bid = a.xmap ? xcd_obj_map(blockIdx.x, gridDim.x, a.tiles) : blockIdx.x;
  const uint32_t obj = bid / a.tiles;
  const uint32_t tile = bid - obj * a.tiles;
  const uint32_t off = packet_lane_off(tile, threadIdx.x, TW, 16u);
  if (off >= a.ps) return;
  const uint64_t o64 = obj;
  __amdgpu_buffer_rsrc_t rs[K];
  uint32_t valid[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    valid[j] = a.in[j].valid;
    rs[j] = shard_rsrc(a.in[j].base, a.in[j].stride, a.in[j].valid, o64, 16u);
  }
  u32x4 acc[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) acc[o] = u32x4{0u, 0u, 0u, 0u};
  cbm_all<BM, D>(acc, rs, valid, a.ps, a.bs, off, std::make_integer_sequence<int, K * 8>{});
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    const DevShard& d = a.out[o / 8];
    const uint32_t pk = (uint32_t)(o % 8) * a.ps;
    uint8_t* p = const_cast<uint8_t*>(d.base) + o64 * d.stride + pk;
    store_guarded(p, off, packet_valid(d.valid, o % 8, a.ps), acc[o]);
  }
}

namespace {

template <class BM, int TW, int WAVES, int D>
int launch_cbm_t(const GfBitApply& p, hipStream_t s) {
  CbmArgs a;
  a.bs = (uint32_t)p.block_size;
  a.ps = (uint32_t)(p.block_size / 8u);
  a.tiles = packet_tiles(a.ps, TW, 16u);
  for (int j = 0; j < kMaxK; ++j)
    a.in[j] = j < BM::K ? dev_shard(p.in[j], 0) : DevShard{nullptr, 0, 0, 0};
  for (int i = 0; i < kMaxR; ++i)
    a.out[i] = i < BM::M ? dev_shard(p.out[i], 0) : DevShard{nullptr, 0, 0, 0};
  a.xmap = (a.tiles <= kObjMapMaxTiles && knobs().gfbit_xmap != 0) ? 1u : 0u;
  const uint64_t grid = p.nobj * a.tiles;
  if (grid == 0 || grid > 0x7FFFFFFFull) return LEOEC_E_ARG;
  hipLaunchKernelGGL((cbm_apply<BM, TW, WAVES, D>), dim3((uint32_t)grid), dim3(TW), 0, s, a);
  return hipGetLastError() == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
}

// the plan's coefficient rows are the compiled matrix's (encode)
template <class BM>
bool is_compiled(const GfBitApply& p) {
  if (p.w != 8 || p.K != BM::K || p.R != BM::M || p.coef.size() != (size_t)BM::K * BM::M)
    return false;
  for (int i = 0; i < BM::M; ++i)
    for (int j = 0; j < BM::K; ++j)
      if (p.coef[(size_t)i * BM::K + j] != BM::m.c[i][j]) return false;
  return true;
}

}  // namespace

// Launches the compiled-schedule kernel if it applies; *rc = its status.
bool launch_cbm(const GfBitApply& p, hipStream_t s, int* rc) {
  const int form = knobs().gfbit_cbm;
  if (form == 0 || !is_compiled<Cbm10_4>(p)) return false;
  if (p.nobj > 0x7FFFFFFFull / 64u || p.block_size >= (1ull << 32)) return false;
  switch (form) {
    case 2: *rc = launch_cbm_t<Cbm10_4, 64, 2, 10>(p, s); return true;
    case 3: *rc = launch_cbm_t<Cbm10_4, 128, 2, 16>(p, s); return true;
    case 4: *rc = launch_cbm_t<Cbm10_4, 64, 3, 4>(p, s); return true;
    case 5: *rc = launch_cbm_t<Cbm10_4, 256, 2, 16>(p, s); return true;
    // round 6: one wave per SIMD (up to 512 VGPRs) with deep look-ahead, the
    // register regime of the 16-byte-lane XOR pattern that read 0.77
    // (tools/packet_ceiling.hip pattern<4,128>: 276 VGPRs, every load of a
    // block pair in flight)
    case 6: *rc = launch_cbm_t<Cbm10_4, 128, 1, 32>(p, s); return true;
    case 7: *rc = launch_cbm_t<Cbm10_4, 64, 1, 32>(p, s); return true;
    case 8: *rc = launch_cbm_t<Cbm10_4, 128, 1, 48>(p, s); return true;
    case 9: *rc = launch_cbm_t<Cbm10_4, 256, 1, 32>(p, s); return true;
    default: *rc = launch_cbm_t<Cbm10_4, 64, 2, 16>(p, s); return true;
  }
}
#endif  // LEOEC_MEASURE

}  // namespace detail
}  // namespace leoec
