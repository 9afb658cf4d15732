// stream_probe.cpp — measurement only: what a HIP stream creation costs, by
// order in the process (the engine's per-thread path creates one stream per
// calling thread and device, engine.cpp get_staging), and whether streams
// created after others were destroyed cost the same.  Each stream runs one
// tiny copy so it is really in use.
//   hipcc --offload-arch=gfx950 -O2 -o tools/stream_probe tools/stream_probe.cpp
//   tools/stream_probe [n]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 8;
  void* d;
  CHECK(hipMalloc(&d, 4096));
  char h[4096] = {0};
  auto use = [&](hipStream_t s) {
    CHECK(hipMemcpyAsync(d, h, sizeof h, hipMemcpyHostToDevice, s));
    CHECK(hipStreamSynchronize(s));
  };
  std::vector<hipStream_t> ss(n);
  for (int i = 0; i < n; ++i) {
    const double t0 = now_ms();
    CHECK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
    const double t1 = now_ms();
    use(ss[i]);
    printf("{\"phase\": \"first %d streams\", \"i\": %d, \"create_ms\": %.3f, \"first_use_ms\": %.3f}\n",
           n, i, t1 - t0, now_ms() - t1);
  }
  for (auto s : ss) CHECK(hipStreamDestroy(s));
  for (int i = 0; i < n; ++i) {
    const double t0 = now_ms();
    CHECK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
    const double t1 = now_ms();
    use(ss[i]);
    printf("{\"phase\": \"after destroying them\", \"i\": %d, \"create_ms\": %.3f, \"first_use_ms\": %.3f}\n",
           i, t1 - t0, now_ms() - t1);
  }
  // streams created on other threads (as dirty schedulers would)
  for (int i = 0; i < 4; ++i) {
    double c = 0, u = 0;
    std::thread t([&] {
      hipStream_t s;
      const double t0 = now_ms();
      CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      const double t1 = now_ms();
      use(s);
      c = t1 - t0;
      u = now_ms() - t1;
      CHECK(hipStreamDestroy(s));
    });
    t.join();
    printf("{\"phase\": \"new thread\", \"i\": %d, \"create_ms\": %.3f, \"first_use_ms\": %.3f}\n", i, c,
           u);
  }
  return 0;
}
