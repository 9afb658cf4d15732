// packet_ceiling.hip — measurement only (not part of the engine): the memory
// ceiling of the cauchyrs(10,4,8) encode's ACCESS PATTERN (gfbit_apply's CEIL
// form: every input packet xor-ed into every output packet, no GF work) on
// the reference's 1 MiB geometry, where packets are ps = 13,120 B (102.5
// cache lines: odd packets start mid line), under variations of the lane
// width, cache policy, object map and boundary handling.
//
// Layout = bench.py's: objects at 1 MiB stride, data block j at j*bs (bs =
// 104,960 = 8 packets), parity in its own buffer at o*4*bs + r*bs.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/packet_ceiling tools/packet_ceiling.hip
//   tools/packet_ceiling [objects] [reps] [object bytes]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int K = 10, R = 4, W = 8;
struct Geo {
  unsigned ps, bs, nobj, tiles;
  unsigned long long obj;
  unsigned omap;  // 1: xcd_obj_map (the engine's, kernels_impl.hpp)
  unsigned k;     // input blocks, at run time (the RT forms' loop bound)
};

__device__ __forceinline__ unsigned obj_map(unsigned b, unsigned n, unsigned tiles) {
  const unsigned full = (n / tiles / 8u) * 8u * tiles;
  if (b >= full) return b;
  const unsigned x = b % 8u, i = b / 8u;
  return ((i / tiles) * 8u + x) * tiles + i % tiles;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, n, 0x00020000);
}

template <int LW>
struct V {
  unsigned v[LW];
};

template <int LW, int LA>
__device__ __forceinline__ V<LW> ld(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  V<LW> r;
  if constexpr (LW == 4) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, LA);
    for (int e = 0; e < 4; ++e) r.v[e] = x[e];
  } else if constexpr (LW == 2) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, LA);
    r.v[0] = x[0];
    r.v[1] = x[1];
  } else {
    r.v[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, LA);
  }
  return r;
}

template <int LW, int SA>
__device__ __forceinline__ void st(const V<LW>& x, __amdgpu_buffer_rsrc_t rs, unsigned off) {
  if constexpr (LW == 4) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(u4{x.v[0], x.v[1], x.v[2], x.v[3]}, rs, off, 0, SA);
  } else if constexpr (LW == 2) {
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u2{x.v[0], x.v[1]}, rs, off, 0, SA);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(x.v[0], rs, off, 0, SA);
  }
}

// One tile = WG lanes x 4*LW bytes of x in every packet.  PF: loads of block
// j+1 in flight while block j is xor-ed in (as gfbit_apply's PFD = 1).
// LA / SA: load / store aux bits (2 = nt).  EDGE: the first and last wave of a
// workgroup load odd packets (the ones that start mid line) with policy 0
// (L2-retained) instead of LA, so the neighbouring tile can hit the shared line;
// EDGE = 2: only the lanes whose bytes lie in the tile's first or last 64 B
// (the half lines an odd packet shares with the neighbouring tiles) do.
template <int LW, int WG, int LA, int SA, int EDGE, int SB = 0>
__global__ void __launch_bounds__(WG) pattern(const unsigned char* __restrict__ in,
                                              unsigned char* __restrict__ out, Geo g) {
  constexpr unsigned LB = 4u * LW;
  const unsigned b = g.omap ? obj_map(blockIdx.x, gridDim.x, g.tiles) : blockIdx.x;
  const unsigned obj = b / g.tiles, tile = b % g.tiles;
  const unsigned off = tile * (WG * LB) + threadIdx.x * LB;
  if (off >= g.ps) return;
  const unsigned in_tile = threadIdx.x * LB;
  const bool edge = EDGE == 1 ? (threadIdx.x / 64u == 0u || threadIdx.x / 64u == WG / 64u - 1u ||
                                 (tile + 1u) * WG * LB > g.ps)
                  : EDGE == 2 ? (in_tile < 64u || in_tile + 64u >= WG * LB || off + 64u >= g.ps)
                              : false;
  const unsigned char* ib = in + (size_t)obj * g.obj;
  unsigned char* ob = out + (size_t)obj * R * g.bs;
  V<LW> acc[R][W];
  for (int i = 0; i < R; ++i)
    for (int x = 0; x < W; ++x)
      for (int e = 0; e < LW; ++e) acc[i][x].v[e] = 0u;
  V<LW> y[2][W];
  auto load = [&](int j, V<LW> (&d)[W]) {
    const auto rs = rsrc(ib + (size_t)j * g.bs, g.bs);
#pragma unroll
    for (int x = 0; x < W; ++x) {
      if (EDGE != 0 && (x & 1) && edge)
        d[x] = ld<LW, 0>(rs, x * g.ps + off);
      else
        d[x] = ld<LW, LA>(rs, x * g.ps + off);
    }
  };
  load(0, y[0]);
  if constexpr (SB) {
    // RT: the engine's shape — a run-time block loop over a 2-slot ring, so
    // the compiler cannot hoist loads or reassociate the XORs across blocks
    auto eat = [&](int j, V<LW> (&d)[W]) {
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int x = 0; x < W; ++x)
#pragma unroll
          for (int e = 0; e < LW; ++e) acc[i][x].v[e] ^= d[x].v[e] + (unsigned)(i * 3 + j);
    };
    const int kk = (int)g.k;
#pragma unroll 1
    for (int j = 0; j < kk; j += 2) {
      if (j + 1 < kk) load(j + 1, y[1]);
      eat(j, y[0]);
      __builtin_amdgcn_sched_barrier(0);
      if (j + 1 >= kk) break;
      if (j + 2 < kk) load(j + 2, y[0]);
      eat(j + 1, y[1]);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j + 1 < K) load(j + 1, y[(j + 1) & 1]);
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int x = 0; x < W; ++x)
#pragma unroll
          for (int e = 0; e < LW; ++e) acc[i][x].v[e] ^= y[j & 1][x].v[e] + (unsigned)(i * 3 + j);
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const auto rs = rsrc(ob + (size_t)i * g.bs, g.bs);
#pragma unroll
    for (int x = 0; x < W; ++x) st<LW, SA>(acc[i][x], rs, x * g.ps + off);
  }
}

// The 8-byte-column register layout of `pattern<2, ...>` (the shipped LW = 2:
// acc 64 VGPRs, ring 32) fed by 16-byte memory instructions.  For packet
// pair (2p, 2p+1) lanes 0-31 of a wave load 16 B of packet 2p and lanes
// 32-63 16 B of packet 2p+1, over the same 512-B span; two
// v_permlane32_swap_b32 per pair (dwords 0<->2, 1<->3, lanes 32-63 of the
// first with lanes 0-31 of the second) then leave lane l holding one 8-byte
// column of BOTH packets: lane l < 32 column 2l, lane l + 32 column 2l + 1.
// Raw loads stay in the ring until the block is consumed (a swap at load
// time would wait on the load).  Stores: the same swaps (an involution),
// then one 16-byte store per pair.  Lanes past the packet load from an
// out-of-range offset (the buffer returns zeros) and do not store.
typedef unsigned u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void swap_pair(unsigned& a, unsigned& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}

template <int WG, int LA, int SA, int SB = 0>
__global__ void __launch_bounds__(WG) pattern_swap(const unsigned char* __restrict__ in,
                                                   unsigned char* __restrict__ out, Geo g) {
  static_assert(W % 2 == 0, "packet pairs");
  const unsigned b = g.omap ? obj_map(blockIdx.x, gridDim.x, g.tiles) : blockIdx.x;
  const unsigned obj = b / g.tiles, tile = b % g.tiles;
  const unsigned lane = threadIdx.x & 63u, half = lane >> 5;
  const unsigned wbase = tile * (WG * 8u) + (threadIdx.x >> 6) * 512u;
  if (wbase >= g.ps) return;  // whole wave past the packet
  const unsigned off = wbase + (lane & 31u) * 16u;
  const bool live = off < g.ps;
  const unsigned char* ib = in + (size_t)obj * g.obj;
  unsigned char* ob = out + (size_t)obj * R * g.bs;
  unsigned acc[R][W][2];
  for (int i = 0; i < R; ++i)
    for (int x = 0; x < W; ++x) acc[i][x][0] = acc[i][x][1] = 0u;
  u4v raw[2][W / 2];
  auto load = [&](int j, u4v (&d)[W / 2]) {
    const auto rs = rsrc(ib + (size_t)j * g.bs, g.bs);
#pragma unroll
    for (int p = 0; p < W / 2; ++p)
      d[p] = __builtin_amdgcn_raw_buffer_load_b128(
          rs, live ? (2u * p + half) * g.ps + off : 0x80000000u, 0, LA);
  };
  auto eat = [&](int j, const u4v (&d)[W / 2]) {
    unsigned y[W][2];
#pragma unroll
    for (int p = 0; p < W / 2; ++p) {
      u4v v = d[p];
      unsigned a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3];
      swap_pair(a0, a2);
      swap_pair(a1, a3);
      y[2 * p][0] = a0;
      y[2 * p][1] = a1;
      y[2 * p + 1][0] = a2;
      y[2 * p + 1][1] = a3;
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int x = 0; x < W; ++x)
#pragma unroll
        for (int e = 0; e < 2; ++e) acc[i][x][e] ^= y[x][e] + (unsigned)(i * 3 + j);
  };
  load(0, raw[0]);
  if constexpr (SB) {  // RT: as pattern<..., SB = 1>
    const int kk = (int)g.k;
#pragma unroll 1
    for (int j = 0; j < kk; j += 2) {
      if (j + 1 < kk) load(j + 1, raw[1]);
      eat(j, raw[0]);
      __builtin_amdgcn_sched_barrier(0);
      if (j + 1 >= kk) break;
      if (j + 2 < kk) load(j + 2, raw[0]);
      eat(j + 1, raw[1]);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j + 1 < K) load(j + 1, raw[(j + 1) & 1]);
      eat(j, raw[j & 1]);
    }
  }
  if (!live) return;  // after the last swap: every lane took part in it
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const auto rs = rsrc(ob + (size_t)i * g.bs, g.bs);
#pragma unroll
    for (int p = 0; p < W / 2; ++p) {
      unsigned a0 = acc[i][2 * p][0], a1 = acc[i][2 * p][1];
      unsigned a2 = acc[i][2 * p + 1][0], a3 = acc[i][2 * p + 1][1];
      swap_pair(a0, a2);
      swap_pair(a1, a3);
      __builtin_amdgcn_raw_buffer_store_b128(u4v{a0, a1, a2, a3}, rs, (2u * p + half) * g.ps + off,
                                             0, SA);
    }
  }
}

__global__ void fill_random(unsigned* p, size_t n, unsigned seed) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned long long z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (unsigned)(z ^ (z >> 31));
  }
}

typedef void (*KFn)(const unsigned char*, unsigned char*, Geo);
struct Case {
  std::string name;
  KFn k;
  unsigned wg, lb, omap;
};
#define KC(LW, WG, LA, SA, E) reinterpret_cast<KFn>(&pattern<LW, WG, LA, SA, (int)(E)>)
#define KS(WG, LA, SA) reinterpret_cast<KFn>(&pattern_swap<WG, LA, SA>)
#define KSB(WG) reinterpret_cast<KFn>(&pattern_swap<WG, 2, 2, 1>)
#define KCB(LW, WG) reinterpret_cast<KFn>(&pattern<LW, WG, 2, 2, 0, 1>)

int main(int argc, char** argv) {
  const unsigned nobj = argc > 1 ? (unsigned)atoi(argv[1]) : 1024u;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const unsigned long long osz = argc > 3 ? strtoull(argv[3], nullptr, 10) : (1ull << 20);
  Geo G{};
  // cauchycoding.cpp geometry, w = 8: bs = ceil16(ceil(N / (k w))) * w, ps = bs / w
  G.bs = (unsigned)(((osz + 8 * K - 1) / (8 * K) + 15) / 16 * 16 * 8);
  G.ps = G.bs / W;
  G.obj = osz;
  G.nobj = nobj;
  G.k = K;
  printf("# object %llu B, bs %u, ps %u (ps mod 128 = %u), %u objects\n", osz, G.bs, G.ps,
         G.ps % 128, nobj);
  unsigned char *in, *out;
  const size_t in_bytes = (size_t)nobj * osz + (size_t)K * G.bs;
  const size_t out_bytes = (size_t)nobj * R * G.bs;
  CHECK(hipMalloc(&in, in_bytes));
  CHECK(hipMalloc(&out, out_bytes));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (unsigned*)in, in_bytes / 4, 7u);
  CHECK(hipMemset(out, 0, out_bytes));
  CHECK(hipDeviceSynchronize());
  const double bytes = (double)nobj * (K + R) * G.bs;
  {
    // the swap forms must produce the 8-byte-lane forms' output exactly (same
    // dword arithmetic, columns only permuted over lanes): one launch each,
    // outputs compared byte for byte
    std::vector<unsigned char> ref(out_bytes), got(out_bytes);
    Geo g = G;
    g.omap = 1;
    g.tiles = (G.ps + 2047u) / 2048u;
    auto run = [&](KFn k, std::vector<unsigned char>& dst) {
      CHECK(hipMemset(out, 0, out_bytes));
      hipLaunchKernelGGL(k, dim3(nobj * g.tiles), dim3(256), 0, 0, in, out, g);
      CHECK(hipMemcpy(dst.data(), out, out_bytes, hipMemcpyDeviceToHost));
    };
    const KFn pairs[2][2] = {{KC(2, 256, 2, 2, 0), KS(256, 2, 2)}, {KCB(2, 256), KSB(256)}};
    for (int q = 0; q < 2; ++q) {
      run(pairs[q][0], ref);
      run(pairs[q][1], got);
      size_t bad = 0;
      for (size_t i = 0; i < out_bytes; ++i) bad += ref[i] != got[i];
      printf("# swap form vs 8-byte-lane form (%s): %zu of %zu output bytes differ\n",
             q ? "run-time K ring" : "unrolled", bad, out_bytes);
      if (bad) return 3;
    }
  }
  std::vector<Case> cases = {
      {"lw8 wg256 nt/nt objmap (shipped shape)", KC(2, 256, 2, 2, false), 256, 8, 1},
      {"swap16 wg256 nt/nt objmap", KS(256, 2, 2), 256, 8, 1},
      {"swap16 wg128 nt/nt objmap", KS(128, 2, 2), 128, 8, 1},
      {"swap16 wg512 nt/nt objmap", KS(512, 2, 2), 512, 8, 1},
      {"swap16 wg256 nt/nt", KS(256, 2, 2), 256, 8, 0},
      {"lw8 wg256 nt/nt objmap ring (run-time K ring)", KCB(2, 256), 256, 8, 1},
      {"swap16 wg256 nt/nt objmap ring (run-time K ring)", KSB(256), 256, 8, 1},
      {"swap16 wg128 nt/nt objmap ring (run-time K ring)", KSB(128), 128, 8, 1},
      {"lw8 wg256 nt/nt objmap edge-waves-L2", KC(2, 256, 2, 2, true), 256, 8, 1},
      {"lw8 wg256 ld0/nt objmap", KC(2, 256, 0, 2, false), 256, 8, 1},
      {"lw8 wg256 sc1nt/nt objmap", KC(2, 256, 18, 2, false), 256, 8, 1},
      {"lw8 wg256 nt/0 objmap", KC(2, 256, 2, 0, false), 256, 8, 1},
      {"lw8 wg128 nt/nt objmap", KC(2, 128, 2, 2, false), 128, 8, 1},
      {"lw8 wg512 nt/nt objmap", KC(2, 512, 2, 2, false), 512, 8, 1},
      {"lw4 wg256 nt/nt objmap", KC(1, 256, 2, 2, false), 256, 4, 1},
      {"lw16 wg256 nt/nt objmap", KC(4, 256, 2, 2, false), 256, 16, 1},
      {"lw16 wg128 nt/nt objmap", KC(4, 128, 2, 2, false), 128, 16, 1},
      {"lw16 wg64 nt/nt objmap", KC(4, 64, 2, 2, false), 64, 16, 1},
      {"lw8 wg256 nt/nt objmap edge-lanes-L2", KC(2, 256, 2, 2, 2), 256, 8, 1},
      {"lw16 wg128 nt/nt objmap edge-waves-L2", KC(4, 128, 2, 2, 1), 128, 16, 1},
      {"lw16 wg128 nt/nt objmap edge-lanes-L2", KC(4, 128, 2, 2, 2), 128, 16, 1},
      {"lw16 wg256 nt/nt objmap edge-lanes-L2", KC(4, 256, 2, 2, 2), 256, 16, 1},
      {"lw16 wg128 nt/nt edge-lanes-L2", KC(4, 128, 2, 2, 2), 128, 16, 0},
  };
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<std::vector<float>> t(cases.size());
  for (int round = 0; round < 4; ++round) {
    for (size_t c = 0; c < cases.size(); ++c) {
      Geo g = G;
      g.omap = cases[c].omap;
      g.tiles = (G.ps + cases[c].wg * cases[c].lb - 1) / (cases[c].wg * cases[c].lb);
      const unsigned grid = nobj * g.tiles;
      auto launch = [&]() {
        hipLaunchKernelGGL(cases[c].k, dim3(grid), dim3(cases[c].wg), 0, 0, in, out, g);
      };
      for (int i = 0; i < 10; ++i) launch();
      for (int i = 0; i < reps; ++i) {
        CHECK(hipEventRecord(a, 0));
        launch();
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        t[c].push_back(ms);
      }
    }
  }
  CHECK(hipGetLastError());
  for (size_t c = 0; c < cases.size(); ++c) {
    std::sort(t[c].begin(), t[c].end());
    const double ms = t[c][t[c].size() / 2];
    printf("{\"case\": \"%s\", \"ms_med\": %.4f, \"frac\": %.4f}\n", cases[c].name.c_str(), ms,
           bytes / ms / 1e6 / 8000.0);
  }
  return 0;
}
