// stream_ceiling.hip — measurement only (not part of the engine): what the
// HBM system gives the RS(10,4,8) 1 MiB encode's ACCESS PATTERN with no GF
// work, under each cache-policy pair, so the shipped kernel's rate can be read
// against its own pattern's ceiling rather than a flat copy.
//
// Layout = bench.py's: 1024 objects at 1 MiB stride, data block j of object o
// at o*1 MiB + j*bs (bs = 104,960), parity in its own buffer at o*4*bs + r*bs.
// One workgroup of 256 lanes per 4 KiB tile of one object (26 tiles per block).
//
// Modes: 0 mixed (10 loads, 4 stores: the encode's traffic, XOR instead of the
// GF product), 1 read-only (the 10 loads, stores predicated off by a runtime
// flag), 2 write-only (the 4 stores), 3 flat copy of the same byte count.
// Cache policy = gfx950 buffer aux bits (1 sc0, 2 nt, 16 sc1).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_ceiling tools/stream_ceiling.hip
//   tools/stream_ceiling [reps] [const|random] [object bytes]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int K = 10, R = 4;
// Geometry (argv[3] = object bytes, default 1 MiB: bs = 104,960, 1024 objects;
// 64 MiB: bs = 6,710,912, 16 objects — BASELINE cfg4).
struct Geo {
  unsigned bs;
  unsigned long long obj;  // object stride
  unsigned nobj;
  unsigned omap;           // 1: the engine's xcd_obj_map (kernels_impl.hpp)
};

// Same remap as the engine: XCD x (ids dealt round-robin) takes objects
// o = x mod 8, each object's tiles in order; ids past the last whole group
// of 8 objects keep their place.
__device__ __forceinline__ unsigned obj_map(unsigned b, unsigned n, unsigned tiles) {
  const unsigned full = (n / tiles / 8u) * 8u * tiles;
  if (b >= full) return b;
  const unsigned x = b % 8u, i = b / 8u;
  return ((i / tiles) * 8u + x) * tiles + i % tiles;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

template <int MODE, int LA, int SA, int CPT = 1, int SEQ = 1, int WG = 256>
__global__ void __launch_bounds__(WG) pattern(const unsigned char* __restrict__ in,
                                              unsigned char* __restrict__ out, int flag, Geo geo) {
  const unsigned BS = geo.bs, NOBJ = geo.nobj;
  const unsigned long long OBJ = geo.obj;
  constexpr unsigned TB = WG * 16u * CPT;                 // bytes of a block per tile
  const unsigned NT = (BS + TB - 1) / TB;                // tiles per block
  for (int q = 0; q < SEQ; ++q) {
    const unsigned g = (SEQ == 1 && geo.omap) ? obj_map(blockIdx.x, gridDim.x, NT) : blockIdx.x * SEQ + q;
    if (g >= NOBJ * NT) return;
    const unsigned obj = g / NT, tile = g % NT;
    const unsigned char* ib = in + (size_t)obj * OBJ;
    unsigned char* ob = out + (size_t)obj * R * BS;
    u32x4 acc[CPT][R];
    unsigned off[CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) off[c] = tile * TB + c * WG * 16u + threadIdx.x * 16u;
    if (MODE != 2) {
      u32x4 d[CPT][K];
#pragma unroll
      for (int j = 0; j < K; ++j)
#pragma unroll
        for (int c = 0; c < CPT; ++c)
          d[c][j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(ib + j * BS), off[c], 0, LA);
#pragma unroll
      for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          acc[c][r] = d[c][r];
#pragma unroll
          for (int j = 0; j < K; ++j)
            if (j != r) acc[c][r] ^= d[c][j];
        }
    } else {
#pragma unroll
      for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[c][r] = u32x4{off[c], obj, (unsigned)r, 0x5a5a5a5au};
    }
    // read-only: a store no real data triggers (the loads stay live)
    if (MODE == 1 && (acc[0][0][0] ^ acc[0][1][1] ^ acc[0][2][2] ^ acc[0][3][3]) != (unsigned)flag + 0x9e3779b9u)
      continue;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int c = 0; c < CPT; ++c)
        if (off[c] < BS)  // buffer stores past num_records are dropped anyway; keep the bound explicit
          __builtin_amdgcn_raw_buffer_store_b128(acc[c][r], rsrc(ob + r * BS), off[c], 0, SA);
  }
}

template <int LA, int SA>
__global__ void __launch_bounds__(256) flat_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b,
                                                 size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(a + (i & ~size_t(0xFFFFF))),
                                                         (unsigned)((i & 0xFFFFF) * 16), 0, LA);
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(b + (i & ~size_t(0xFFFFF))),
                                         (unsigned)((i & 0xFFFFF) * 16), 0, SA);
}

__global__ void fill_random(unsigned* p, size_t n, unsigned seed) {  // splitmix-style hash
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned long long z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (unsigned)(z ^ (z >> 31));
  }
}

struct Case {
  const char* name;
  void (*k)(const unsigned char*, unsigned char*, int, Geo);
  double bytes;  // algorithmic bytes per launch
  unsigned grid, wg;
  unsigned omap = 0;
};

#define PATX(M, L, S, C, Q, W) reinterpret_cast<void (*)(const unsigned char*, unsigned char*, int, Geo)>(&pattern<M, L, S, C, Q, W>)
#define PAT(M, L, S) PATX(M, L, S, 1, 1, 256)
static Geo G;
unsigned grid_of(unsigned cpt, unsigned seq, unsigned wg) {
  return (G.nobj * ((G.bs + wg * 16u * cpt - 1) / (wg * 16u * cpt)) + seq - 1) / seq;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const unsigned long long osz = argc > 3 ? strtoull(argv[3], nullptr, 10) : (1ull << 20);
  // leo_erasure geometry (c_src/common.cpp:24-33, rscoding.cpp:44), w = 8:
  // bs = ceil16(ceil(N / (k w))) * w  (a multiple of 128: whole cache lines)
  G.bs = (unsigned)(((osz + 8 * K - 1) / (8 * K) + 15) / 16 * 16 * 8);
  G.obj = osz;
  G.nobj = (unsigned)((1ull << 30) / osz);
  G.omap = 0;
  const unsigned BS = G.bs, NOBJ = G.nobj;
  const unsigned long long OBJ = G.obj;
  printf("# object %llu B, bs %u, %u objects\n", OBJ, BS, NOBJ);
  unsigned char *in, *out;
  const double rd = (double)NOBJ * K * BS, wr = (double)NOBJ * R * BS;
  const size_t ncopy = (size_t)((rd + wr) / 2 / 16);  // flat copy: same bytes moved as the pattern
  // both buffers hold the pattern's footprint and the flat copy's (the copy
  // moves (rd + wr) / 2 bytes each way, more than the parity buffer)
  const size_t in_bytes = std::max((size_t)(NOBJ * OBJ + (size_t)K * BS), ncopy * 16);
  const size_t out_bytes = std::max((size_t)NOBJ * R * BS, ncopy * 16);
  CHECK(hipMalloc(&in, in_bytes));
  CHECK(hipMalloc(&out, out_bytes));
  // argv[2] == "const": constant bytes (0x37); default: pseudo-random bytes
  if (argc > 2 && argv[2][0] == 'c') CHECK(hipMemset(in, 0x37, in_bytes));
  else hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (unsigned*)in, in_bytes / 4, 7u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemset(out, 0, out_bytes));
  std::vector<Case> cases = {
      {"mixed ld=nt st=nt", PAT(0, 2, 2), rd + wr, grid_of(1, 1, 256), 256},
      {"mixed ld=0 st=0", PAT(0, 0, 0), rd + wr, grid_of(1, 1, 256), 256},
      {"mixed ld=nt st=0", PAT(0, 2, 0), rd + wr, grid_of(1, 1, 256), 256},
      {"mixed ld=0 st=nt", PAT(0, 0, 2), rd + wr, grid_of(1, 1, 256), 256},
      {"mixed ld=nt st=sc0sc1nt", PAT(0, 2, 19), rd + wr, grid_of(1, 1, 256), 256},
      {"mixed ld=sc1nt st=nt", PAT(0, 18, 2), rd + wr, grid_of(1, 1, 256), 256},
      {"mixed ld=sc0nt st=nt", PAT(0, 3, 2), rd + wr, grid_of(1, 1, 256), 256},
      {"mixed ld=sc1 st=sc1", PAT(0, 16, 16), rd + wr, grid_of(1, 1, 256), 256},
      {"read-only ld=nt", PAT(1, 2, 2), rd, grid_of(1, 1, 256), 256},
      {"read-only ld=0", PAT(1, 0, 0), rd, grid_of(1, 1, 256), 256},
      {"write-only st=nt", PAT(2, 2, 2), wr, grid_of(1, 1, 256), 256},
      {"write-only st=0", PAT(2, 0, 0), wr, grid_of(1, 1, 256), 256},
      {"mixed nt cpt2", PATX(0, 2, 2, 2, 1, 256), rd + wr, grid_of(2, 1, 256), 256},
      {"mixed nt seq2", PATX(0, 2, 2, 1, 2, 256), rd + wr, grid_of(1, 2, 256), 256},
      {"mixed nt seq4", PATX(0, 2, 2, 1, 4, 256), rd + wr, grid_of(1, 4, 256), 256},
      {"mixed nt wg64", PATX(0, 2, 2, 1, 1, 64), rd + wr, grid_of(1, 1, 64), 64},
      {"mixed nt wg128", PATX(0, 2, 2, 1, 1, 128), rd + wr, grid_of(1, 1, 128), 128},
      {"mixed nt wg512", PATX(0, 2, 2, 1, 1, 512), rd + wr, grid_of(1, 1, 512), 512},
      {"mixed nt wg64 cpt4", PATX(0, 2, 2, 4, 1, 64), rd + wr, grid_of(4, 1, 64), 64},
  };
  const size_t nbase = cases.size();
  for (size_t c = 0; c < nbase; ++c)  // every single-tile case again under the object map
    if (cases[c].grid == grid_of(1, 1, cases[c].wg) && std::string(cases[c].name).find("seq") == std::string::npos) {
      Case m = cases[c];
      m.omap = 1;
      m.name = strdup((std::string(m.name) + " objmap").c_str());
      cases.push_back(m);
    }
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<std::vector<float>> t(cases.size() + 2);
  for (int round = 0; round < 5; ++round) {
    for (size_t c = 0; c < cases.size() + 2; ++c) {
      auto launch = [&]() {
        if (c < cases.size())
          {
          Geo g = G;
          g.omap = cases[c].omap;
          hipLaunchKernelGGL(cases[c].k, dim3(cases[c].grid), dim3(cases[c].wg), 0, 0, in, out, 0, g);
        }
        else if (c == cases.size())
          hipLaunchKernelGGL((flat_copy<2, 2>), dim3((unsigned)((ncopy + 255) / 256)), dim3(256), 0, 0,
                             (const u32x4*)in, (u32x4*)out, ncopy);
        else
          hipLaunchKernelGGL((flat_copy<0, 0>), dim3((unsigned)((ncopy + 255) / 256)), dim3(256), 0, 0,
                             (const u32x4*)in, (u32x4*)out, ncopy);
      };
      for (int i = 0; i < 40; ++i) launch();  // warm (>= 10 ms of launches)
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
  for (size_t c = 0; c < cases.size() + 2; ++c) {
    std::sort(t[c].begin(), t[c].end());
    const double ms = t[c][t[c].size() / 2];
    const char* name = c < cases.size() ? cases[c].name : (c == cases.size() ? "flat copy nt" : "flat copy");
    const double bytes = c < cases.size() ? cases[c].bytes : rd + wr;
    printf("{\"case\": \"%s\", \"ms_med\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n", name, ms,
           bytes / ms / 1e6, bytes / ms / 1e6 / 8000.0);
  }
  return 0;
}
