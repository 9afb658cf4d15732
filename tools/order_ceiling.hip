// order_ceiling.hip — measurement only (not part of the engine): how the
// workgroup -> (object, tile) ORDER changes what HBM gives the RS(10,4,8)
// encode's access pattern (10 loads + 4 stores per column, XOR instead of the
// GF product, nt/nt policy as shipped), for large objects (BASELINE cfg4:
// 64 MiB objects, bs 6,710,912) and, for reference, 1 MiB objects.
//
// Layout = bench.py's: objects at obj stride, data block j of object o at
// o*obj + j*bs; parity in its own buffer at o*4*bs + r*bs.
//
// Orders (g = workgroup id after the optional XCD remap):
//   0 tile-major         obj = g / T, tile = g % T           (engine default > 64 tiles)
//   1 object-major       tile = g / N, obj = g % N
//   2 chunked            chunks of C tiles, objects interleaved per chunk:
//                        g -> (chunk q, obj o, i) = C-tile segment q of object o
//   3 xcd objects        XCD x takes objects o = x mod 8, tile-major inside (xcd_obj_map)
//   4 xcd segments       XCD x takes tile segment x of every object (8 segments/object),
//                        objects in turn, tiles in order inside a segment
//   5 xcd chunked        as 2, but the 8 XCDs each own 1/8 of each chunk row:
//                        XCD x takes the C-tile chunks (q, o) with (q*N + o) % 8 == x
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/order_ceiling tools/order_ceiling.hip
//   tools/order_ceiling [object bytes] [objects] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int K = 10, R = 4;
struct Geo {
  unsigned bs;
  unsigned long long spacing;  // bytes from data block j to j+1 (bs = the reference's layout)
  unsigned long long obj;
  unsigned nobj;
  unsigned tiles;  // tiles per block
  unsigned order, chunk;
  unsigned skew;  // diagnostic: blocks K/2..K-1 read `skew` bytes further along than blocks 0..K/2-1
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

// grid n = N*T ids; the dispatcher deals ids round-robin over the 8 XCDs, so
// id b runs on XCD b % 8 as its (b / 8)-th workgroup there.
__device__ __forceinline__ void place(unsigned b, unsigned n, const Geo& g, unsigned& obj,
                                      unsigned& tile) {
  const unsigned N = g.nobj, T = g.tiles, C = g.chunk;
  switch (g.order) {
    case 1: tile = b / N; obj = b % N; return;
    case 2: {  // chunk rows: all objects' chunk q, then chunk q+1 (ragged last chunk:
               // ids past the block exit)
      const unsigned row = b / (C * N), r = b % (C * N);
      obj = r / C;
      tile = row * C + r % C;
      return;
    }
    case 3: {
      const unsigned full = (n / T / 8u) * 8u * T;
      unsigned m = b;
      if (b < full) {
        const unsigned x = b % 8u, i = b / 8u;
        m = ((i / T) * 8u + x) * T + i % T;
      }
      obj = m / T;
      tile = m % T;
      return;
    }
    case 4: {  // needs T % 8 == 0 handled: segment length S = ceil(T/8), last short
      const unsigned x = b % 8u, i = b / 8u;          // XCD, its i-th workgroup
      const unsigned S = (T + 7u) / 8u;
      // XCD x owns tiles [x*S, min(T,(x+1)*S)) of every object
      const unsigned lo = x * S, hi = min(T, lo + S), len = hi > lo ? hi - lo : 0u;
      if (len == 0u || i >= len * N) {  // spill (ragged segments): fall back to identity
        obj = b / T;
        tile = b % T;
        return;
      }
      obj = i / len;
      tile = lo + i % len;
      return;
    }
    case 5: {  // chunks (q, o) in row-major order dealt round-robin over the XCDs
      const unsigned x = b % 8u, i = b / 8u;
      const unsigned ch = (i / C) * 8u + x;
      obj = ch % N;
      tile = (ch / N) * C + i % C;
      if (ch / N >= (T + C - 1) / C) tile = T;  // padding id: exits
      return;
    }
    default: obj = b / T; tile = b % T; return;
  }
}

template <int WG>
__global__ void __launch_bounds__(WG) pattern(const unsigned char* __restrict__ in,
                                              unsigned char* __restrict__ out, Geo geo) {
  unsigned obj, tile;
  place(blockIdx.x, gridDim.x, geo, obj, tile);
  const unsigned BS = geo.bs;
  const unsigned char* ib = in + (size_t)obj * geo.obj;
  unsigned char* ob = out + (size_t)obj * R * BS;
  if (tile >= geo.tiles || obj >= geo.nobj) return;
  const unsigned off = tile * (WG * 16u) + threadIdx.x * 16u;
  if (off >= BS) return;
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    // (skew: a pattern experiment, the XOR then mixes columns — not a code)
    // skew 1: the 1 KiB windows of a pair swap (off ^ 1024), else a shift
    const unsigned o = j >= K / 2 && geo.skew
                           ? (geo.skew == 1u ? ((off ^ 1024u) < BS ? off ^ 1024u : off) : (off + geo.skew) % BS)
                           : off;
    d[j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(ib + (size_t)j * geo.spacing), o, 0, 2);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    u32x4 acc = d[r];
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (j != r) acc ^= d[j];
    __builtin_amdgcn_raw_buffer_store_b128(acc, rsrc(ob + (size_t)r * BS), off, 0, 2);
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

struct Case {
  std::string name;
  unsigned wg, order, chunk;
};

int main(int argc, char** argv) {
  const unsigned long long osz = argc > 1 ? strtoull(argv[1], nullptr, 10) : (64ull << 20);
  const unsigned nobj = argc > 2 ? (unsigned)atoi(argv[2]) : 64u;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  // diagnostic only (argv[4]): extra bytes between consecutive data blocks,
  // i.e. NOT the reference's layout; argv[5] = "quick": tile-major orders only
  const unsigned long long pad = argc > 4 ? strtoull(argv[4], nullptr, 10) : 0ull;
  const bool quick = argc > 5 && std::string(argv[5]) == "quick";
  const unsigned skew = argc > 6 ? (unsigned)strtoul(argv[6], nullptr, 10) : 0u;
  Geo G{};
  G.bs = (unsigned)(((osz + 8 * K - 1) / (8 * K) + 15) / 16 * 16 * 8);
  G.spacing = G.bs + pad;
  G.skew = skew;
  if (skew) printf("# blocks %d..%d read %u bytes further along (pattern experiment)\n", K / 2, K - 1, skew);
  G.obj = pad ? (unsigned long long)K * G.spacing : osz;
  G.nobj = nobj;
  printf("# object %llu B, bs %u, block spacing %llu, %u objects\n", osz, G.bs, G.spacing, nobj);
  unsigned char *in, *out;
  const size_t in_bytes = (size_t)nobj * G.obj + (size_t)K * G.spacing;
  const size_t out_bytes = (size_t)nobj * R * G.bs;
  CHECK(hipMalloc(&in, in_bytes));
  CHECK(hipMalloc(&out, out_bytes));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (unsigned*)in, in_bytes / 4, 7u);
  CHECK(hipMemset(out, 0, out_bytes));
  CHECK(hipDeviceSynchronize());
  const double bytes = (double)nobj * (K + R) * G.bs;
  std::vector<Case> cases;
  for (unsigned wg : {64u, 256u}) {
    const std::string w = " wg" + std::to_string(wg);
    cases.push_back({"tile-major" + w, wg, 0, 1});
    if (quick) continue;
    cases.push_back({"object-major" + w, wg, 1, 1});
    cases.push_back({"xcd objects" + w, wg, 3, 1});
    cases.push_back({"xcd segments" + w, wg, 4, 1});
    for (unsigned c : {8u, 26u, 64u, 128u, 256u, 512u, 1024u}) {
      cases.push_back({"chunked C" + std::to_string(c) + w, wg, 2, c});
      cases.push_back({"xcd chunked C" + std::to_string(c) + w, wg, 5, c});
    }
  }
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<std::vector<float>> t(cases.size());
  std::vector<bool> skip(cases.size(), false);
  for (int round = 0; round < 3; ++round) {
    for (size_t c = 0; c < cases.size(); ++c) {
      Geo g = G;
      g.tiles = (G.bs + cases[c].wg * 16u - 1) / (cases[c].wg * 16u);
      g.order = cases[c].order;
      g.chunk = cases[c].chunk;
      if ((g.order == 2 || g.order == 5) && g.chunk > g.tiles) { skip[c] = true; continue; }
      unsigned grid = nobj * g.tiles;
      if (g.order == 2 || g.order == 5) {  // whole chunks (and, for 5, whole rounds of 8)
        const unsigned nch = ((g.tiles + g.chunk - 1) / g.chunk) * nobj;
        grid = (g.order == 5 ? (nch + 7u) / 8u * 8u : nch) * g.chunk;
      }
      auto launch = [&]() {
        if (cases[c].wg == 64)
          hipLaunchKernelGGL(pattern<64>, dim3(grid), dim3(64), 0, 0, in, out, g);
        else
          hipLaunchKernelGGL(pattern<256>, dim3(grid), dim3(256), 0, 0, in, out, g);
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
    if (skip[c] || t[c].empty()) continue;
    std::sort(t[c].begin(), t[c].end());
    const double ms = t[c][t[c].size() / 2];
    printf("{\"case\": \"%s\", \"ms_med\": %.4f, \"frac\": %.4f}\n", cases[c].name.c_str(), ms,
           bytes / ms / 1e6 / 8000.0);
  }
  return 0;
}
