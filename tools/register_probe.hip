// register_probe.hip — measurement only (not part of the engine): what a
// lone caller's 1 MiB call could save by pinning the caller's memory in
// place instead of packing it.  The per-thread zero-copy path today packs the
// object into a pinned, device-mapped buffer (a host copy of the whole
// object) and unpacks the parity from it; the kernel reads / writes that
// buffer over PCIe.  This times, per object size, on the system runtime:
//   pack      memcpy of the object into a hipHostMalloc'd mapped buffer
//   register  hipHostRegister (mapped) + hipHostGetDevicePointer +
//             hipHostUnregister of the caller's (malloc'ed, touched) buffer,
//             the same buffer every time and a different one every time
//   read      a kernel reading the object over PCIe (zero-copy) from the
//             mapped buffer and from the registered caller memory
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/register_probe tools/register_probe.hip
//   tools/register_probe [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

__global__ void __launch_bounds__(256) read16(const u4* __restrict__ src, u4* __restrict__ dst,
                                              size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dst[i] = __builtin_nontemporal_load(src + i);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  CHECK(hipSetDevice(0));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t maxb = (size_t)4 << 20;
  unsigned char *mapped, *mapped_d, *dev;
  CHECK(hipHostMalloc((void**)&mapped, maxb, hipHostMallocMapped));
  CHECK(hipHostGetDevicePointer((void**)&mapped_d, mapped, 0));
  CHECK(hipMalloc((void**)&dev, maxb));
  // a pool of caller buffers (page-aligned like a large malloc)
  constexpr int kPool = 64;
  std::vector<unsigned char*> pool(kPool);
  for (auto& p : pool) {
    if (posix_memalign((void**)&p, 4096, maxb)) return 1;
    memset(p, 0x5A, maxb);
  }
  for (size_t bytes : {(size_t)256 << 10, (size_t)1 << 20, (size_t)4 << 20}) {
    std::vector<double> pack, reg_same, reg_new, rd_mapped, rd_reg;
    const size_t n16 = bytes / 16;
    const unsigned grid = 256;
    for (int r = 0; r < reps; ++r) {
      unsigned char* src = pool[r % kPool];
      double t0 = now_us();
      memcpy(mapped, src, bytes);
      pack.push_back(now_us() - t0);
      // register the same buffer every time
      t0 = now_us();
      CHECK(hipHostRegister(pool[0], bytes, hipHostRegisterMapped));
      void* d = nullptr;
      CHECK(hipHostGetDevicePointer(&d, pool[0], 0));
      CHECK(hipHostUnregister(pool[0]));
      reg_same.push_back(now_us() - t0);
      // a different buffer every time (as an Erlang binary would be)
      t0 = now_us();
      CHECK(hipHostRegister(src, bytes, hipHostRegisterMapped));
      CHECK(hipHostGetDevicePointer(&d, src, 0));
      const double t_reg = now_us() - t0;
      // the kernel reading it over PCIe
      double t1 = now_us();
      hipLaunchKernelGGL(read16, dim3(grid), dim3(256), 0, s, (const u4*)d, (u4*)dev, n16);
      CHECK(hipStreamSynchronize(s));
      rd_reg.push_back(now_us() - t1);
      t1 = now_us();
      CHECK(hipHostUnregister(src));
      reg_new.push_back(t_reg + now_us() - t1);
      t1 = now_us();
      hipLaunchKernelGGL(read16, dim3(grid), dim3(256), 0, s, (const u4*)mapped_d, (u4*)dev, n16);
      CHECK(hipStreamSynchronize(s));
      rd_mapped.push_back(now_us() - t1);
    }
    printf("{\"bytes\": %zu, \"pack_us\": %.1f, \"register_same_us\": %.1f, \"register_new_us\": %.1f, "
           "\"read_mapped_us\": %.1f, \"read_registered_us\": %.1f}\n",
           bytes, median(pack), median(reg_same), median(reg_new), median(rd_mapped), median(rd_reg));
    fflush(stdout);
  }
  return 0;
}
