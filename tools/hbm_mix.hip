// hbm_mix.hip — measurement only (not part of the engine): what HBM gives the
// headline's byte stream when its reads and its writes run alone.  RS(10,4,8)
// at 1 MiB: per object 10 input blocks of bs = 104,960 B in a row of 10 bs,
// 4 output blocks in a row of 4 bs (bench.py's layout); one workgroup of 256
// lanes per 4 KiB column tile of an object, 16 B per lane, non-temporal, the
// engine's object-interleaved XCD order.  Kernels:
//   mix      read 10 blocks, xor, write 4 (the encode's traffic, no GF math)
//   read10   the 10 reads alone (the xor stored only if it equals a value it
//            never takes, so nothing is written)
//   write4   the 4 writes alone
//   read14   14 blocks read (the mix's byte count, all reads)
//   write14  14 blocks written
// If mix takes about read10 + write4, the encode's rate is the read and write
// rates of the part and the mix costs nothing; if it takes longer, the
// turnaround between them does.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_mix tools/hbm_mix.hip
//   tools/hbm_mix [objects] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
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

typedef unsigned u4 __attribute__((ext_vector_type(4)));
constexpr unsigned kBs = 104960, kTile = 4096, kTiles = (kBs + kTile - 1) / kTile;

// the engine's xcd_obj_map: XCD x (workgroup ids dealt round robin) takes
// objects o = x mod 8, all tiles of one object in order
__device__ __forceinline__ unsigned obj_map(unsigned b, unsigned n) {
  const unsigned full = (n / kTiles / 8u) * 8u * kTiles;
  if (b >= full) return b;
  const unsigned x = b % 8u, i = b / 8u;
  return ((i / kTiles) * 8u + x) * kTiles + i % kTiles;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

// LPOL / SPOL: the cache-policy bits of the loads / stores (raw buffer
// instructions' aux operand on gfx950: 1 sc0, 2 nt, 16 sc1; 2 = the engine's)
template <int NR, int NW, bool XOR, int LPOL = 2, int SPOL = 2>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8)))
stream(const unsigned char* __restrict__ in, unsigned char* __restrict__ out, unsigned long long irow,
       unsigned long long orow, unsigned never) {
  const unsigned b = obj_map(blockIdx.x, gridDim.x);
  const unsigned obj = b / kTiles, tile = b % kTiles;
  const unsigned off = tile * kTile + threadIdx.x * 16u;
  if (off >= kBs) return;
  u4 a = {threadIdx.x, obj, tile, 7u};
  const auto ir = rsrc(in + (size_t)obj * irow);
  u4 v[NR > 0 ? NR : 1];
#pragma unroll
  for (int j = 0; j < NR; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(ir, j * kBs + off, 0, LPOL);
#pragma unroll
  for (int j = 0; j < NR; ++j) a ^= v[j];
  const auto orr = rsrc(out + (size_t)obj * orow);
  if (NW == 0) {
    if (a.x == never && a.y == never) __builtin_amdgcn_raw_buffer_store_b128(a, orr, off, 0, SPOL);
    return;
  }
#pragma unroll
  for (int r = 0; r < NW; ++r) {
    u4 o = a;
    if (XOR) o.w ^= (unsigned)r;
    __builtin_amdgcn_raw_buffer_store_b128(o, orr, r * kBs + off, 0, SPOL);
  }
}

__global__ void fill(unsigned* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    p[i] = (unsigned)(i * 2654435761u) ^ 0x5bd1e995u;
}

typedef void (*KFn)(const unsigned char*, unsigned char*, unsigned long long, unsigned long long,
                    unsigned);

int main(int argc, char** argv) {
  const unsigned n = argc > 1 ? (unsigned)atoi(argv[1]) : 2048u;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const unsigned long long irow = 14ull * kBs, orow = 14ull * kBs;
  const size_t bytes = (size_t)n * irow + 4096;
  unsigned char *in, *out;
  CHECK(hipMalloc(&in, bytes));
  CHECK(hipMalloc(&out, bytes));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (unsigned*)in, bytes / 4);
  CHECK(hipDeviceSynchronize());
  struct Case {
    const char* name;
    KFn k;
    int reads, writes;
    unsigned long long ir, orr;
  };
  // read rows of 10 bs / write rows of 4 bs as the bench; the 14-block forms
  // at rows of 14 bs
  const unsigned long long R10 = 10ull * kBs, R4 = 4ull * kBs, R14 = 14ull * kBs;
  const std::vector<Case> cases = {
      {"mix: read 10, write 4", &stream<10, 4, true>, 10, 4, R10, R4},
      {"read10", &stream<10, 0, false>, 10, 0, R10, R4},
      {"write4", &stream<0, 4, true>, 0, 4, R10, R4},
      {"read14", &stream<14, 0, false>, 14, 0, R14, R4},
      {"write14", &stream<0, 14, true>, 0, 14, R10, R14},
      {"read10, loads plain", &stream<10, 0, false, 0>, 10, 0, R10, R4},
      {"read10, loads sc0", &stream<10, 0, false, 1>, 10, 0, R10, R4},
      {"write4, stores plain", &stream<0, 4, true, 2, 0>, 0, 4, R10, R4},
      {"write4, stores sc0", &stream<0, 4, true, 2, 1>, 0, 4, R10, R4},
      {"write4, stores sc0 nt", &stream<0, 4, true, 2, 3>, 0, 4, R10, R4},
      {"write4, stores sc1", &stream<0, 4, true, 2, 16>, 0, 4, R10, R4},
      {"write4, stores sc1 nt", &stream<0, 4, true, 2, 18>, 0, 4, R10, R4},
      {"write4, stores sc0 sc1", &stream<0, 4, true, 2, 17>, 0, 4, R10, R4},
      {"mix, stores plain", &stream<10, 4, true, 2, 0>, 10, 4, R10, R4},
      {"mix, stores sc1 nt", &stream<10, 4, true, 2, 18>, 10, 4, R10, R4},
      {"mix, loads plain, stores plain", &stream<10, 4, true, 0, 0>, 10, 4, R10, R4},
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(cases.size());
  const unsigned grid = n * kTiles;
  for (int round = 0; round < 3; ++round) {
    for (size_t c = 0; c < cases.size(); ++c) {
      const Case& cs = cases[c];
      auto launch = [&]() {
        hipLaunchKernelGGL(cs.k, dim3(grid), dim3(256), 0, 0, in, out, cs.ir, cs.orr, 0xdeadbeefu);
      };
      {  // time-based warm-up: clocks ramp over the first milliseconds
        CHECK(hipEventRecord(e0, 0));
        float ms = 0.f;
        while (ms < 200.f) {
          for (int i = 0; i < 10; ++i) launch();
          CHECK(hipEventRecord(e1, 0));
          CHECK(hipEventSynchronize(e1));
          CHECK(hipEventElapsedTime(&ms, e0, e1));
        }
      }
      for (int i = 0; i < reps; ++i) {
        CHECK(hipEventRecord(e0, 0));
        launch();
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t[c].push_back(ms);
      }
    }
  }
  CHECK(hipGetLastError());
  std::vector<double> med(cases.size());
  for (size_t c = 0; c < cases.size(); ++c) {
    std::sort(t[c].begin(), t[c].end());
    med[c] = t[c][t[c].size() / 2];
    const double b = (double)n * (cases[c].reads + cases[c].writes) * kBs;
    printf("{\"case\": \"%s\", \"objects\": %u, \"ms_med\": %.4f, \"TBps\": %.3f, \"frac\": %.4f}\n",
           cases[c].name, n, med[c], b / med[c] / 1e9, b / med[c] / 1e9 / 8.0);
  }
  const double b14 = (double)n * 14 * kBs;
  printf("{\"case\": \"read10 + write4 back to back (sum of times)\", \"ms\": %.4f, \"frac\": %.4f, "
         "\"mix_over_sum\": %.4f}\n",
         med[1] + med[2], b14 / (med[1] + med[2]) / 1e9 / 8.0, med[0] / (med[1] + med[2]));
  CHECK(hipFree(in));
  CHECK(hipFree(out));
  return 0;
}
