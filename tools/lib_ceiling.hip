// lib_ceiling.hip — measurement only (not part of the engine): the memory
// ceiling of the liberation(k,2,w) encode's ACCESS PATTERN on the
// reference's 1 MiB geometry (round-5 verdict item 1).  liberation(7,2,7):
// block bs = 149,856 B = 7 packets of ps = 21,408 B (167.25 cache lines:
// packet x of block j starts 32 * ((7 j + x) mod 4) bytes into a 128-B
// line), objects in rows of k * bs, P and Q in their own buffer.
//
// Every form reads each input packet once and writes each output packet
// once, 16 bytes per lane, XOR instead of the liberation structure (every
// input packet x of every block into P[x] and Q[x]), so the arithmetic is
// nothing; the forms differ in how loads are issued:
//   branchy  the shipped lib_apply's shape: a per-load uniform branch
//            between a plain load and a guarded one (every load then waits
//            for all outstanding loads), packet ring of LA
//   ring     raw buffer loads, no branch, LA packets in flight (libb_apply)
//   block    raw buffer loads, a whole block (w packets) in flight
//   copy     a plain streaming copy-and-XOR of the same bytes: each lane
//            reads its 16 B of the k data blocks' flat rows and writes 2
//            blocks' worth, no packet structure (the part's rate for this
//            byte count)
// on the reference geometry and on objects sized so packets are line
// aligned (ps = 21,504 B), at 64 and 256 lanes per workgroup; then the
// syndrome decode's access (dec_pattern: decode of data blocks {0,1}).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/lib_ceiling tools/lib_ceiling.hip
//   tools/lib_ceiling [objects] [reps] [k] [decode-form]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
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

constexpr int W = 7;
typedef unsigned u4 __attribute__((ext_vector_type(4)));

struct Geo {
  unsigned ps, bs, tiles, k;
  unsigned long long row;  // object row bytes (k * bs)
  unsigned full_tiles;     // tiles wholly inside the packet
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
__device__ __forceinline__ void pin(u4& v) { asm volatile("" : "+v"(v)); }

// FORM 0 branchy, 1 ring, 2 block.  K compiled in (the engine's libb form).
template <int K, int FORM, int LA, int TW>
__global__ void __launch_bounds__(TW) __attribute__((amdgpu_waves_per_eu(4, 8)))
pattern(const unsigned char* __restrict__ in, unsigned char* __restrict__ out, Geo g) {
  const unsigned b = obj_map(blockIdx.x, gridDim.x, g.tiles);
  const unsigned obj = b / g.tiles, tile = b % g.tiles;
  const unsigned t0 = tile * TW * 16u, off = t0 + threadIdx.x * 16u;
  const bool full = tile < g.full_tiles;  // wave-uniform
  const unsigned char* ib = in + (size_t)obj * g.row;
  unsigned char* ob = out + (size_t)obj * 2 * g.bs;
  u4 P[W], Q[W];
  for (int x = 0; x < W; ++x) P[x] = Q[x] = u4{0u, 0u, 0u, 0u};
  auto load = [&](int q) -> u4 {
    const int j = q / W, x = q % W;
    const unsigned pos = (unsigned)x * g.ps + off;
    if constexpr (FORM == 0) {
      const unsigned char* p = ib + (size_t)j * g.bs + pos;
      if (full) return __builtin_nontemporal_load(reinterpret_cast<const u4*>(p));
      u4 v = {0u, 0u, 0u, 0u};
      if (off < g.ps) v = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p));
      return v;
    } else {
      return __builtin_amdgcn_raw_buffer_load_b128(rsrc(ib + (size_t)j * g.bs, g.bs), pos, 0, 2);
    }
  };
  auto eat = [&](int q, u4 v) {
    const int x = q % W;
    P[x] ^= v;
    Q[x] ^= v;
    if constexpr (FORM != 0) {
      pin(P[x]);
      pin(Q[x]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  constexpr int NP = K * W;
  if constexpr (FORM == 2) {
    u4 y[2][W];
#pragma unroll
    for (int x = 0; x < W; ++x) y[0][x] = load(x);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j + 1 < K)
#pragma unroll
        for (int x = 0; x < W; ++x) y[(j + 1) & 1][x] = load((j + 1) * W + x);
#pragma unroll
      for (int x = 0; x < W; ++x) eat(j * W + x, y[j & 1][x]);
    }
  } else {
    constexpr int RS = LA + 1;
    u4 ring[RS];
#pragma unroll
    for (int q = 0; q < LA; ++q) ring[q] = load(q);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if (p + LA < NP) ring[(p + LA) % RS] = load(p + LA);
      eat(p, ring[p % RS]);
    }
  }
  if (off >= g.ps) return;
#pragma unroll
  for (int x = 0; x < W; ++x) {
    unsigned char* p = ob + (size_t)x * g.ps + off;
    __builtin_nontemporal_store(P[x], reinterpret_cast<u4*>(p));
    __builtin_nontemporal_store(Q[x], reinterpret_cast<u4*>(p + g.bs));
  }
}

// FORM sweep (round 5, session 33): line-aligned loads with the packets'
// misalignment undone in the lanes.  A 64-lane wave sweeps ST consecutive
// 1 KiB tiles of every packet.  Packet q (block j, packet x) starts delta_q
// = (address mod 128) bytes into a line; its tile t needs the bytes
// [t*1024, +1024) = V_t[delta:] ++ V_{t+1}[:delta] of the LINE-ALIGNED
// windows V_t = [start - delta + t*1024, +1024): each window is loaded once
// (8 lines, not 9), the previous one kept in VGPRs (`carry`), and the lane
// rotation by delta / 16 lanes goes through a 2 KiB LDS scratch (ds_write of
// both windows, ds_read at the offset; one wave per workgroup, so in order
// without a barrier).  LA: packets of look-ahead for the next windows.
template <int K, int ST, int LA>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 8)))
sweep(const unsigned char* __restrict__ in, unsigned char* __restrict__ out, Geo g) {
  constexpr int NP = K * W;
  __shared__ u4 scratch[128];
  const unsigned nsw = (g.tiles + ST - 1) / ST;
  const unsigned b = obj_map(blockIdx.x, gridDim.x, nsw);
  const unsigned obj = b / nsw, sw = b % nsw;
  const unsigned tb = sw * ST, te = tb + ST < g.tiles ? tb + ST : g.tiles;
  const unsigned lane = threadIdx.x;
  const unsigned char* ib = in + (size_t)obj * g.row;
  unsigned char* ob = out + (size_t)obj * 2 * g.bs;
  // per packet: its line-aligned start (as an offset in the object row,
  // which starts on a line) and its shift in 16-B lanes
  auto aligned_at = [&](int q) -> unsigned {
    const unsigned a = (unsigned)(q / W) * g.bs + (unsigned)(q % W) * g.ps;
    return a & ~127u;
  };
  auto shift = [&](int q) -> unsigned {
    const unsigned a = (unsigned)(q / W) * g.bs + (unsigned)(q % W) * g.ps;
    return (a & 127u) / 16u;
  };
  const auto rs = rsrc(ib, (unsigned)g.row);  // past the row: zeros
  auto load = [&](int q, unsigned t) -> u4 {
    return __builtin_amdgcn_raw_buffer_load_b128(rs, aligned_at(q) + t * 1024u + lane * 16u, 0, 2);
  };
  u4 carry[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) carry[q] = load(q, tb);
  for (unsigned t = tb; t < te; ++t) {
    u4 P[W], Q[W];
#pragma unroll
    for (int x = 0; x < W; ++x) P[x] = Q[x] = u4{0u, 0u, 0u, 0u};
    u4 ring[LA + 1];
#pragma unroll
    for (int q = 0; q < LA; ++q) ring[q] = load(q, t + 1);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      if (q + LA < NP) ring[(q + LA) % (LA + 1)] = load(q + LA, t + 1);
      const u4 nxt = ring[q % (LA + 1)];
      scratch[lane] = carry[q];
      scratch[64 + lane] = nxt;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      const u4 v = scratch[lane + shift(q)];
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      carry[q] = nxt;
      const int x = q % W;
      P[x] ^= v;
      Q[x] ^= v;
      pin(P[x]);
      pin(Q[x]);
    }
    const unsigned off = t * 1024u + lane * 16u;
    if (off < g.ps) {
#pragma unroll
      for (int x = 0; x < W; ++x) {
        unsigned char* p = ob + (size_t)x * g.ps + off;
        __builtin_nontemporal_store(P[x], reinterpret_cast<u4*>(p));
        __builtin_nontemporal_store(Q[x], reinterpret_cast<u4*>(p + g.bs));
      }
    }
  }
}

// Decode {0,1} (round 6, verdict r5 item 5): the access of the syndrome
// decode libb_dec_apply — one packet stream P (W packets), Q (W), then data
// blocks 0..K-1, with data blocks 0 and 1 erased (their loads return zeros
// through an empty buffer resource, no memory access) and LA packets in
// flight — but the body only XORs: every packet into both output blocks'
// packet x (no syndrome structure, no mask combine).  Inputs: the K - 2
// surviving data blocks in the object row, P and Q in the parity buffer
// (objects' 2 blocks each); outputs: data blocks 0 and 1 in the object row,
// as the engine's device decode writes them.
//   LA > 0  the shipped stream (zeros for the absent blocks)
//   LA = 0  the block form: absent blocks skipped by a uniform branch, a
//           present block's W loads in flight together
//   PRESENT the ring over the present blocks only (P, Q, D2..): the stream
//           the shipped kernel would have if its absent blocks cost nothing
template <int K, int LA, int TW, bool PRESENT>
__global__ void __launch_bounds__(TW) __attribute__((amdgpu_waves_per_eu(4, 8)))
dec_pattern(unsigned char* __restrict__ rows, const unsigned char* __restrict__ par, Geo g) {
  const unsigned b = obj_map(blockIdx.x, gridDim.x, g.tiles);
  const unsigned obj = b / g.tiles, tile = b % g.tiles;
  const unsigned off = tile * TW * 16u + threadIdx.x * 16u;
  unsigned char* ib = rows + (size_t)obj * g.row;
  const unsigned char* pb = par + (size_t)obj * 2 * g.bs;
  // stream block s: 0 P, 1 Q, 2 + j data j (0, 1 erased: empty resource)
  auto rs = [&](int s) {
    if (s < 2) return rsrc(pb + (size_t)s * g.bs, g.bs);
    return rsrc(ib + (size_t)(s - 2) * g.bs, s - 2 < 2 ? 0u : g.bs);
  };
  u4 A[W], B[W];
  for (int x = 0; x < W; ++x) A[x] = B[x] = u4{0u, 0u, 0u, 0u};
  auto eat = [&](int x, u4 v) {
    A[x] ^= v;
    B[x] ^= v;
    pin(A[x]);
    pin(B[x]);
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int NB = K + 2;
  if constexpr (PRESENT) {
    // present blocks: stream positions 0, 1, 4, 5, .. (P, Q, D2, ..)
    constexpr int NPB = NB - 2, NP = NPB * W, RS = LA + 1;
    auto blk = [](int i) { return i < 2 ? i : i + 2; };
    u4 ring[RS];
#pragma unroll
    for (int q = 0; q < LA; ++q)
      ring[q] = __builtin_amdgcn_raw_buffer_load_b128(rs(blk(q / W)), (unsigned)(q % W) * g.ps + off, 0, 2);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int q = p + LA;
      if (q < NP)
        ring[q % RS] = __builtin_amdgcn_raw_buffer_load_b128(rs(blk(q / W)), (unsigned)(q % W) * g.ps + off, 0, 2);
      eat(p % W, ring[p % RS]);
    }
  } else if constexpr (LA == 0) {
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      if (s == 2 || s == 3) continue;  // the erased blocks: a uniform skip
      const auto r = rs(s);
      u4 y[W];
#pragma unroll
      for (int x = 0; x < W; ++x) y[x] = __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)x * g.ps + off, 0, 2);
#pragma unroll
      for (int x = 0; x < W; ++x) eat(x, y[x]);
    }
  } else {
    constexpr int NP = NB * W, RS = LA + 1;
    u4 ring[RS];
#pragma unroll
    for (int q = 0; q < LA; ++q)
      ring[q] = __builtin_amdgcn_raw_buffer_load_b128(rs(q / W), (unsigned)(q % W) * g.ps + off, 0, 2);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int q = p + LA;
      if (q < NP) ring[q % RS] = __builtin_amdgcn_raw_buffer_load_b128(rs(q / W), (unsigned)(q % W) * g.ps + off, 0, 2);
      eat(p % W, ring[p % RS]);
    }
  }
  if (off >= g.ps) return;
#pragma unroll
  for (int x = 0; x < W; ++x) {
    __builtin_nontemporal_store(A[x], reinterpret_cast<u4*>(ib + (size_t)x * g.ps + off));
    __builtin_nontemporal_store(B[x], reinterpret_cast<u4*>(ib + g.bs + (size_t)x * g.ps + off));
  }
}

// A flat streaming kernel over the same bytes: lane l of tile t reads 16 B
// at t * TW * 16 + l * 16 of each of the K data blocks (blocks as flat
// rows, no packets) and writes the XOR to both output blocks.
template <int K, int TW>
__global__ void __launch_bounds__(TW) __attribute__((amdgpu_waves_per_eu(4, 8)))
flat(const unsigned char* __restrict__ in, unsigned char* __restrict__ out, Geo g,
     unsigned ftiles) {
  const unsigned b = obj_map(blockIdx.x, gridDim.x, ftiles);
  const unsigned obj = b / ftiles, tile = b % ftiles;
  const unsigned off = tile * TW * 16u + threadIdx.x * 16u;
  if (off >= g.bs) return;
  const unsigned char* ib = in + (size_t)obj * g.row;
  u4 a = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < K; ++j)
    a ^= __builtin_nontemporal_load(reinterpret_cast<const u4*>(ib + (size_t)j * g.bs + off));
  unsigned char* ob = out + (size_t)obj * 2 * g.bs;
  __builtin_nontemporal_store(a, reinterpret_cast<u4*>(ob + off));
  __builtin_nontemporal_store(a, reinterpret_cast<u4*>(ob + g.bs + off));
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
  unsigned tw;
  bool aligned;
  unsigned st = 0;  // sweep form: tiles per wave (grid = objects x ceil(tiles / st))
};

// only >= 0: launch decode form `only` `reps` times and nothing else (a
// target for rocprofv3 --pmc passes: tools/pmc_r6_libdec.sh)
template <int K>
int run(unsigned nobj, int reps, int only) {
  // liberation geometry (engine op_layout): bs = ceil16(ceil(N / (k w))) * w
  auto geo = [&](unsigned long long osz) {
    Geo g{};
    const unsigned long long per = (osz + (unsigned long long)K * W - 1) / ((unsigned long long)K * W);
    g.bs = (unsigned)((per + 15) / 16 * 16 * W);
    g.ps = g.bs / W;
    g.k = K;
    g.row = (unsigned long long)K * g.bs;
    return g;
  };
  const Geo ref = geo(1ull << 20);
  // line-aligned packets: ps rounded up to 128
  const unsigned long long apacket = (ref.ps + 127) / 128 * 128;
  const Geo ali = geo(apacket * W * K);
  printf("# liberation(%d,2,%d), %u objects: ps %u (mod 128 = %u), aligned ps %u (mod 128 = %u)\n",
         K, W, nobj, ref.ps, ref.ps % 128, ali.ps, ali.ps % 128);
  const size_t in_bytes = (size_t)nobj * ali.row + 4096, out_bytes = (size_t)nobj * 2 * ali.bs + 4096;
  unsigned char *in, *out, *out2;
  CHECK(hipMalloc(&in, in_bytes));
  CHECK(hipMalloc(&out, out_bytes));
  CHECK(hipMalloc(&out2, out_bytes));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (unsigned*)in, in_bytes / 4, 7u);
  CHECK(hipDeviceSynchronize());
#define PC(F, LA, TW) reinterpret_cast<KFn>(&pattern<K, F, LA, TW>)
#define SW(ST, LA) reinterpret_cast<KFn>(&sweep<K, ST, LA>)
  std::vector<Case> cases = {
      {"branchy la2 wg64 (shipped lib_apply's load shape)", PC(0, 2, 64), 64, false},
      {"ring la2 wg64 (libb_apply)", PC(1, 2, 64), 64, false},
      {"ring la4 wg64", PC(1, 4, 64), 64, false},
      {"ring la8 wg64", PC(1, 8, 64), 64, false},
      {"block wg64", PC(2, 0, 64), 64, false},
      {"ring la2 wg256", PC(1, 2, 256), 256, false},
      {"ring la4 wg256", PC(1, 4, 256), 256, false},
      {"block wg256", PC(2, 0, 256), 256, false},
      {"branchy la2 wg64, aligned packets", PC(0, 2, 64), 64, true},
      {"ring la2 wg64, aligned packets", PC(1, 2, 64), 64, true},
      {"ring la4 wg64, aligned packets", PC(1, 4, 64), 64, true},
      {"block wg64, aligned packets", PC(2, 0, 64), 64, true},
      {"sweep 4 tiles la2 (aligned loads, lanes rotated via LDS)", SW(4, 2), 64, false, 4},
      {"sweep 8 tiles la2", SW(8, 2), 64, false, 8},
      {"sweep 8 tiles la4", SW(8, 4), 64, false, 8},
      {"sweep 16 tiles la2", SW(16, 2), 64, false, 16},
  };
  // every packet form computes the same XORs: outputs compared with the
  // first form's, byte for byte, on the reference geometry
  if (only < 0) {
    std::vector<unsigned char> a(out_bytes), b(out_bytes);
    for (size_t c = 0; c < cases.size(); ++c) {
      if (cases[c].aligned) continue;
      Geo g = ref;
      g.tiles = (g.ps + cases[c].tw * 16 - 1) / (cases[c].tw * 16);
      g.full_tiles = g.ps / (cases[c].tw * 16);
      const unsigned grid = cases[c].st ? (g.tiles + cases[c].st - 1) / cases[c].st : g.tiles;
      CHECK(hipMemset(out, 0, out_bytes));
      hipLaunchKernelGGL(cases[c].k, dim3(nobj * grid), dim3(cases[c].tw), 0, 0, in, out, g);
      CHECK(hipMemcpy(c == 0 ? a.data() : b.data(), out, out_bytes, hipMemcpyDeviceToHost));
      if (c && a != b) {
        printf("# form %s: output differs from the branchy form\n", cases[c].name.c_str());
        return 3;
      }
    }
    printf("# every reference-geometry form wrote the same bytes\n");
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(cases.size() + 2);
  for (int round = 0; round < (only < 0 ? 4 : 0); ++round) {
    for (size_t c = 0; c < cases.size() + 2; ++c) {
      Geo g = c < cases.size() && cases[c].aligned ? ali : ref;
      std::function<void()> launch;
      if (c < cases.size()) {
        g.tiles = (g.ps + cases[c].tw * 16 - 1) / (cases[c].tw * 16);
        g.full_tiles = g.ps / (cases[c].tw * 16);
        const KFn k = cases[c].k;
        const unsigned tw = cases[c].tw;
        const unsigned grid = cases[c].st ? (g.tiles + cases[c].st - 1) / cases[c].st : g.tiles;
        launch = [=]() { hipLaunchKernelGGL(k, dim3(nobj * grid), dim3(tw), 0, 0, in, out, g); };
      } else {
        const unsigned tw = c == cases.size() ? 64 : 256;
        const unsigned ft = (g.bs + tw * 16 - 1) / (tw * 16);
        launch = [=]() {
          if (tw == 64) hipLaunchKernelGGL((flat<K, 64>), dim3(nobj * ft), dim3(64), 0, 0, in, out2, g, ft);
          else hipLaunchKernelGGL((flat<K, 256>), dim3(nobj * ft), dim3(256), 0, 0, in, out2, g, ft);
        };
      }
      {  // time-based warm-up: the clock ramps over the first milliseconds
        CHECK(hipEventRecord(e0, 0));
        float ms = 0.f;
        while (ms < 300.f) {
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
  for (size_t c = 0; only < 0 && c < cases.size() + 2; ++c) {
    std::sort(t[c].begin(), t[c].end());
    const double ms = t[c][t[c].size() / 2];
    const Geo g = c < cases.size() && cases[c].aligned ? ali : ref;
    const double bytes = (double)nobj * (K + 2) * g.bs;
    const std::string name = c < cases.size() ? cases[c].name
                             : c == cases.size() ? "flat copy-xor wg64 (same bytes, no packets)"
                                                 : "flat copy-xor wg256 (same bytes, no packets)";
    printf("{\"k\": %d, \"case\": \"%s\", \"ms_med\": %.4f, \"frac\": %.4f}\n", K, name.c_str(), ms,
           bytes / ms / 1e6 / 8000.0);
  }
  // decode {0,1}: the stream forms on the reference geometry, outputs (data
  // blocks 0 and 1 of every object row) compared byte for byte; the parity
  // buffer is `out` (its first 2 blocks per object), left as the encode
  // forms wrote it
  {
    typedef void (*DFn)(unsigned char*, const unsigned char*, Geo);
    struct DCase {
      std::string name;
      DFn k;
      unsigned tw;
    };
#define DC(LA, TW, PR) reinterpret_cast<DFn>(&dec_pattern<K, LA, TW, PR>)
    std::vector<DCase> dcases = {
        {"decode {0,1}: stream la4 wg64 (shipped libb_dec_apply's access at k <= 4)", DC(4, 64, false), 64},
        {"decode {0,1}: stream la2 wg64 (shipped at k >= 5, w <= 11)", DC(2, 64, false), 64},
        {"decode {0,1}: block form wg64 (absent blocks skipped)", DC(0, 64, false), 64},
        {"decode {0,1}: present blocks only, la4 wg64", DC(4, 64, true), 64},
        {"decode {0,1}: present blocks only, la8 wg64", DC(8, 64, true), 64},
        {"decode {0,1}: stream la4 wg256", DC(4, 256, false), 256},
    };
    Geo g = ref;
    if (only >= 0) {
      if (only >= (int)dcases.size()) return 4;
      g.tiles = (g.ps + dcases[only].tw * 16 - 1) / (dcases[only].tw * 16);
      for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(dcases[only].k, dim3(nobj * g.tiles), dim3(dcases[only].tw), 0, 0, in, out, g);
      CHECK(hipDeviceSynchronize());
      printf("# decode form %s: %d launches\n", dcases[only].name.c_str(), reps);
      return 0;
    }
    std::vector<unsigned char> a((size_t)nobj * g.row), b((size_t)nobj * g.row);
    for (size_t c = 0; c < dcases.size(); ++c) {
      g.tiles = (g.ps + dcases[c].tw * 16 - 1) / (dcases[c].tw * 16);
      CHECK(hipMemset(in, 0, (size_t)nobj * g.row));  // D0, D1 rewritten, the rest zero
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, (unsigned*)in, (size_t)nobj * g.row / 4, 9u);
      hipLaunchKernelGGL(dcases[c].k, dim3(nobj * g.tiles), dim3(dcases[c].tw), 0, 0, in, out, g);
      CHECK(hipMemcpy(c == 0 ? a.data() : b.data(), in, a.size(), hipMemcpyDeviceToHost));
      if (c && a != b) {
        printf("# decode form %s: output differs from the first decode form\n", dcases[c].name.c_str());
        return 3;
      }
    }
    printf("# every decode form wrote the same bytes\n");
    std::vector<std::vector<float>> dt(dcases.size());
    for (int round = 0; round < 4; ++round) {
      for (size_t c = 0; c < dcases.size(); ++c) {
        g.tiles = (g.ps + dcases[c].tw * 16 - 1) / (dcases[c].tw * 16);
        const DFn kf = dcases[c].k;
        const unsigned tw = dcases[c].tw;
        auto launch = [=]() { hipLaunchKernelGGL(kf, dim3(nobj * g.tiles), dim3(tw), 0, 0, in, out, g); };
        CHECK(hipEventRecord(e0, 0));
        float ms = 0.f;
        while (ms < 300.f) {
          for (int i = 0; i < 10; ++i) launch();
          CHECK(hipEventRecord(e1, 0));
          CHECK(hipEventSynchronize(e1));
          CHECK(hipEventElapsedTime(&ms, e0, e1));
        }
        for (int i = 0; i < reps; ++i) {
          CHECK(hipEventRecord(e0, 0));
          launch();
          CHECK(hipEventRecord(e1, 0));
          CHECK(hipEventSynchronize(e1));
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          dt[c].push_back(ms);
        }
      }
    }
    CHECK(hipGetLastError());
    for (size_t c = 0; c < dcases.size(); ++c) {
      std::sort(dt[c].begin(), dt[c].end());
      const double ms = dt[c][dt[c].size() / 2];
      const double bytes = (double)nobj * (K + 2) * g.bs;  // K survivors in, 2 blocks out
      printf("{\"k\": %d, \"case\": \"%s\", \"ms_med\": %.4f, \"frac\": %.4f}\n", K,
             dcases[c].name.c_str(), ms, bytes / ms / 1e6 / 8000.0);
    }
  }
  CHECK(hipFree(in));
  CHECK(hipFree(out));
  CHECK(hipFree(out2));
  return 0;
}

int main(int argc, char** argv) {
  const unsigned nobj = argc > 1 ? (unsigned)atoi(argv[1]) : 1024u;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int k = argc > 3 ? atoi(argv[3]) : 7;
  const int only = argc > 4 ? atoi(argv[4]) : -1;  // a decode form alone (PMC target)
  if (k == 4) return run<4>(nobj, reps, only);
  return run<7>(nobj, reps, only);
}
