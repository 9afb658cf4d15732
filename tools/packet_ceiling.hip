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
template <int LW, int WG, int LA, int SA, int EDGE>
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
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const auto rs = rsrc(ob + (size_t)i * g.bs, g.bs);
#pragma unroll
    for (int x = 0; x < W; ++x) st<LW, SA>(acc[i][x], rs, x * g.ps + off);
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
  std::vector<Case> cases = {
      {"lw8 wg256 nt/nt", KC(2, 256, 2, 2, false), 256, 8, 0},
      {"lw8 wg256 nt/nt objmap", KC(2, 256, 2, 2, false), 256, 8, 1},
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
