// duplex_probe.hip — measurement only (not part of the engine): can the host
// path's two directions share the PCIe link at once?
//
// The bench's link leg (bench.py `host_path.link`, a torch process) read
// 56.8 GB/s H2D alone, 56.4 D2H alone and 56.5 GB/s for BOTH at once on two
// streams, and the batching queue's `link_busy` 1.01, as if the link's two
// directions could not overlap.  This probe times each direction moved by
// the DMA engines (hipMemcpyAsync) and by a kernel (CUs loading from /
// storing to pinned, device-mapped host memory), alone and in every pairing
// at once, and the queue's copy shape (per-slot streams against one H2D and
// one D2H stream), from plain C++ on the system runtime.  Found
// (profiles/r05_s18_duplex_*.log, r05_s19_duplex_queue.log): two DMA copies
// on separate streams overlap (97 GB/s together); the queue's per-slot form
// moved 44.8 GB/s, the two-stream form 73.4, which the queue now uses
// (hostq.cpp launch_slot).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/duplex_probe tools/duplex_probe.hip
//   tools/duplex_probe [MiB per direction] [reps] [kernel workgroups]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

// Grid-stride copy, 16 B per lane, 4 loads in flight per lane.  NT = 1:
// non-temporal loads and stores.
template <int NT>
__global__ void __launch_bounds__(256) copy16(const u4* __restrict__ src, u4* __restrict__ dst,
                                              size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    u4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

__global__ void fill(unsigned* p, size_t n, unsigned seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = (unsigned)(i * 2654435761u) ^ seed;
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 256;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int wgs = argc > 3 ? atoi(argv[3]) : 512;
  const size_t bytes = mib << 20, n16 = bytes / 16;
  CHECK(hipSetDevice(0));
  unsigned char *hin, *hout, *din, *dout, *hin_d, *hout_d;
  CHECK(hipHostMalloc((void**)&hin, bytes, hipHostMallocMapped));
  CHECK(hipHostMalloc((void**)&hout, bytes, hipHostMallocMapped));
  CHECK(hipHostGetDevicePointer((void**)&hin_d, hin, 0));
  CHECK(hipHostGetDevicePointer((void**)&hout_d, hout, 0));
  CHECK(hipMalloc((void**)&din, bytes));
  CHECK(hipMalloc((void**)&dout, bytes));
  for (size_t i = 0; i < bytes; i += 4096) hin[i] = (unsigned char)i, hout[i] = 0;
  memset(hin, 0x5A, bytes);
  memset(hout, 0, bytes);
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, (unsigned*)dout, bytes / 4, 7u);
  CHECK(hipDeviceSynchronize());
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));

  // the four movers: one direction each, on a given stream
  auto dma_h2d = [&](hipStream_t s) { CHECK(hipMemcpyAsync(din, hin, bytes, hipMemcpyHostToDevice, s)); };
  auto dma_d2h = [&](hipStream_t s) { CHECK(hipMemcpyAsync(hout, dout, bytes, hipMemcpyDeviceToHost, s)); };
  auto krn_h2d = [&](hipStream_t s) {
    hipLaunchKernelGGL(copy16<1>, dim3(wgs), dim3(256), 0, s, (const u4*)hin_d, (u4*)din, n16);
  };
  auto krn_d2h = [&](hipStream_t s) {
    hipLaunchKernelGGL(copy16<1>, dim3(wgs), dim3(256), 0, s, (const u4*)dout, (u4*)hout_d, n16);
  };
  struct Case {
    std::string name;
    std::function<void()> run;
    int dirs;  // directions moved (bytes = dirs * size)
  };
  std::vector<Case> cases = {
      {"dma h2d", [&] { dma_h2d(s1); }, 1},
      {"dma d2h", [&] { dma_d2h(s2); }, 1},
      {"dma h2d + dma d2h", [&] { dma_h2d(s1); dma_d2h(s2); }, 2},
      {"kernel h2d", [&] { krn_h2d(s1); }, 1},
      {"kernel d2h", [&] { krn_d2h(s2); }, 1},
      {"kernel h2d + dma d2h", [&] { krn_h2d(s1); dma_d2h(s2); }, 2},
      {"dma h2d + kernel d2h", [&] { dma_h2d(s1); krn_d2h(s2); }, 2},
      {"kernel h2d + kernel d2h", [&] { krn_h2d(s1); krn_d2h(s2); }, 2},
  };
  // The batching queue's shape (hostq.cpp launch_slot): batches of a 16 MiB
  // input arena in and a 6.4 MiB output arena out (RS(10,4): 0.4 of the
  // input), 5 slots, each slot's H2D and D2H in order on its own stream;
  // against the same batches with every H2D on one stream and every D2H on
  // another (each D2H after its batch's H2D through an event).
  constexpr int kSlots = 5, kBatches = 40;
  const size_t bin = (size_t)16 << 20, bout = bin * 2 / 5;
  hipStream_t ss[kSlots];
  hipEvent_t evs[kBatches];
  for (auto& x : ss) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  for (auto& e : evs) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  auto slot_in = [&](int b) { return (size_t)(b % kSlots) * bin; };
  auto slot_out = [&](int b) { return (size_t)(b % kSlots) * bout; };
  cases.push_back({"queue shape: 5 slot streams, H2D + D2H per slot", [&] {
                     for (int b = 0; b < kBatches; ++b) {
                       hipStream_t st = ss[b % kSlots];
                       CHECK(hipMemcpyAsync(din + slot_in(b), hin + slot_in(b), bin, hipMemcpyHostToDevice, st));
                       CHECK(hipMemcpyAsync(hout + slot_out(b), dout + slot_out(b), bout, hipMemcpyDeviceToHost, st));
                     }
                   }, -1});
  cases.push_back({"queue shape: H2D stream + D2H stream", [&] {
                     for (int b = 0; b < kBatches; ++b) {
                       CHECK(hipMemcpyAsync(din + slot_in(b), hin + slot_in(b), bin, hipMemcpyHostToDevice, s1));
                       CHECK(hipEventRecord(evs[b], s1));
                       CHECK(hipStreamWaitEvent(s2, evs[b], 0));
                       CHECK(hipMemcpyAsync(hout + slot_out(b), dout + slot_out(b), bout, hipMemcpyDeviceToHost, s2));
                     }
                   }, -1});
  cases.push_back({"queue shape: H2D alone", [&] {
                     for (int b = 0; b < kBatches; ++b)
                       CHECK(hipMemcpyAsync(din + slot_in(b), hin + slot_in(b), bin, hipMemcpyHostToDevice, s1));
                   }, -2});
  // Caller memory (an Erlang binary is pageable): the same pair of copies
  // from / to malloc'ed memory as is (the runtime stages it) and pinned in
  // place with hipHostRegister.
  unsigned char *pin_in = nullptr, *pin_out = nullptr, *pg_in = nullptr, *pg_out = nullptr;
  if (posix_memalign((void**)&pin_in, 4096, bytes) || posix_memalign((void**)&pin_out, 4096, bytes) ||
      posix_memalign((void**)&pg_in, 4096, bytes) || posix_memalign((void**)&pg_out, 4096, bytes))
    return 1;
  memset(pin_in, 0x5A, bytes);
  memset(pin_out, 0, bytes);
  memset(pg_in, 0x5A, bytes);
  memset(pg_out, 0, bytes);
  CHECK(hipHostRegister(pin_in, bytes, hipHostRegisterDefault));
  CHECK(hipHostRegister(pin_out, bytes, hipHostRegisterDefault));
  cases.push_back({"registered h2d", [&] { CHECK(hipMemcpyAsync(din, pin_in, bytes, hipMemcpyHostToDevice, s1)); }, 1});
  cases.push_back({"registered h2d + registered d2h", [&] {
                     CHECK(hipMemcpyAsync(din, pin_in, bytes, hipMemcpyHostToDevice, s1));
                     CHECK(hipMemcpyAsync(pin_out, dout, bytes, hipMemcpyDeviceToHost, s2));
                   }, 2});
  cases.push_back({"pageable h2d", [&] { CHECK(hipMemcpyAsync(din, pg_in, bytes, hipMemcpyHostToDevice, s1)); }, 1});
  cases.push_back({"pageable d2h", [&] { CHECK(hipMemcpyAsync(pg_out, dout, bytes, hipMemcpyDeviceToHost, s2)); }, 1});
  cases.push_back({"pageable h2d + pageable d2h", [&] {
                     CHECK(hipMemcpyAsync(din, pg_in, bytes, hipMemcpyHostToDevice, s1));
                     CHECK(hipMemcpyAsync(pg_out, dout, bytes, hipMemcpyDeviceToHost, s2));
                   }, 2});
  // 8 chunks of 32 MiB from registered memory: each chunk's H2D on s1, its
  // D2H on s2 after an event (the shape of a column-chunked large call)
  constexpr int kCh = 8;
  hipEvent_t ch_ev[kCh];
  for (auto& e : ch_ev) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  cases.push_back({"registered, 8 chunks: h2d(c) || d2h(c-1)", [&] {
                     const size_t cb = bytes / kCh;
                     for (int c = 0; c < kCh; ++c) {
                       CHECK(hipMemcpyAsync(din + c * cb, pin_in + c * cb, cb, hipMemcpyHostToDevice, s1));
                       CHECK(hipEventRecord(ch_ev[c], s1));
                       CHECK(hipStreamWaitEvent(s2, ch_ev[c], 0));
                       CHECK(hipMemcpyAsync(pin_out + c * cb, dout + c * cb, cb, hipMemcpyDeviceToHost, s2));
                     }
                   }, 2});
  printf("# %zu MiB per direction, %d reps, kernel grid %d x 256 lanes\n", mib, reps, wgs);
  for (auto& c : cases) {
    c.run();  // warm-up
    CHECK(hipDeviceSynchronize());
    std::vector<double> ms;
    for (int r = 0; r < reps; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      c.run();
      CHECK(hipDeviceSynchronize());
      ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    if (c.dirs < 0) {  // the queue shapes: batches of bin in (and bout out)
      const double in_b = (double)kBatches * bin, out_b = c.dirs == -1 ? (double)kBatches * bout : 0.0;
      printf("{\"case\": \"%s\", \"ms_med\": %.3f, \"GBps_total\": %.1f, \"GBps_h2d\": %.1f}\n",
             c.name.c_str(), med, (in_b + out_b) / med / 1e6, in_b / med / 1e6);
      fflush(stdout);
      continue;
    }
    printf("{\"case\": \"%s\", \"ms_med\": %.3f, \"GBps_total\": %.1f, \"GBps_per_direction\": %.1f}\n",
           c.name.c_str(), med, c.dirs * (double)bytes / med / 1e6, (double)bytes / med / 1e6);
    fflush(stdout);
  }
  // the copies moved the right bytes
  CHECK(hipMemcpy(hout, dout, 4096, hipMemcpyDeviceToHost));
  std::vector<unsigned char> chk(4096);
  CHECK(hipMemcpy(chk.data(), din, 4096, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int i = 0; i < 4096; ++i) ok = ok && chk[i] == 0x5A;
  printf("{\"h2d_bytes_ok\": %s}\n", ok ? "true" : "false");
  return ok ? 0 : 1;
}
