// large_copy_probe.cpp — measurement only (not part of the engine): how the
// host<->device copies of ONE large object can be arranged, for the host
// path of objects above 16 MiB (the reference's own benchmark encodes one
// 100 MiB binary: test/leo_erasure_tests.erl:207-212, 331-336).
//
// The engine's per-thread path today: one pageable H2D of the object, the
// kernel, one pageable D2H of the m coding blocks — the D2H cannot start
// before the H2D ends.  A GF(2^w) code is column-separable (parity bytes
// [c0, c1) of every coding block depend only on bytes [c0, c1) of every data
// block), so the object can move in C column chunks with chunk c's parity
// D2H overlapping chunk c+1's H2D on the full-duplex link.  This probe times
// the copies alone (the kernel of a 100 MiB object is ~30 us) in the
// arrangements such a path could use, each from ordinary malloc'ed
// (pageable, touched) host memory:
//
//   serial           H2D of the object, then D2H of the parity (today's copies)
//   serial-reg       the same after hipHostRegister of both host ranges
//   chunk2d-C        C chunks, hipMemcpy2DAsync k rows (pitch bs) in, m rows out,
//                    D2H of chunk c on a second stream after chunk c's H2D
//   chunk2d-reg-C    the same on registered host memory (register + unregister
//                    inside the timed region)
//   chunk1d-reg-C    registered, one 1-D copy per block segment (k in, m out)
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/large_copy_probe tools/large_copy_probe.cpp
//   tools/large_copy_probe [object MiB] [reps]
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

static double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 100;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int k = 10, m = 4, w = 8;
  const size_t size = mib << 20;
  // rscoding.cpp:44 geometry
  const size_t bs = ((size + (size_t)k * w - 1) / ((size_t)k * w) + 15) / 16 * 16 * w;
  uint8_t* src = static_cast<uint8_t*>(malloc((size_t)k * bs));
  uint8_t* out = static_cast<uint8_t*>(malloc((size_t)m * bs));
  memset(src, 1, (size_t)k * bs);  // touched, as an Erlang binary is
  memset(out, 2, (size_t)m * bs);
  uint8_t* dev;
  CHECK(hipMalloc(&dev, (size_t)(k + m) * bs));
  hipStream_t sa, sb;
  {  // the first stream of the process sets up the device's hardware queues
    const double t0 = now_ms();
    CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    const double t1 = now_ms();
    CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    const double t2 = now_ms();
    printf("{\"case\": \"hipStreamCreate\", \"first_ms\": %.3f, \"second_ms\": %.3f}\n", t1 - t0,
           t2 - t1);
  }
  std::vector<hipEvent_t> ev(64);
  for (auto& e : ev) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  printf("# object %zu MiB, k %d m %d, bs %zu; host link bytes %zu\n", mib, k, m, bs,
         (size_t)k * bs + (size_t)m * bs);

  {  // the first pageable copies of the process, and of these buffers
    const double t0 = now_ms();
    CHECK(hipMemcpy(dev, src, (size_t)k * bs, hipMemcpyHostToDevice));
    const double t1 = now_ms();
    CHECK(hipMemcpy(dev, src, (size_t)k * bs, hipMemcpyHostToDevice));
    const double t2 = now_ms();
    printf("{\"case\": \"pageable H2D of the object, first / second\", \"first_ms\": %.3f, "
           "\"second_ms\": %.3f}\n", t1 - t0, t2 - t1);
  }
  const bool poison = argc > 3 && std::string(argv[3]) == "poison";
  auto reg = [&](bool on) {
    if (on) {
      CHECK(hipHostRegister(src, (size_t)k * bs, hipHostRegisterDefault));
      CHECK(hipHostRegister(out, (size_t)m * bs, hipHostRegisterDefault));
    } else {
      CHECK(hipHostUnregister(src));
      CHECK(hipHostUnregister(out));
    }
  };
  auto serial = [&](bool r) {
    if (r) reg(true);
    CHECK(hipMemcpyAsync(dev, src, (size_t)k * bs, hipMemcpyHostToDevice, sa));
    CHECK(hipMemcpyAsync(out, dev + (size_t)k * bs, (size_t)m * bs, hipMemcpyDeviceToHost, sa));
    CHECK(hipStreamSynchronize(sa));
    if (r) reg(false);
  };
  auto chunked = [&](int C, bool r, bool twod) {
    if (r) reg(true);
    const size_t cw = (bs / C + 15) / 16 * 16;
    int c = 0;
    for (size_t c0 = 0; c0 < bs; c0 += cw, ++c) {
      const size_t n = std::min(cw, bs - c0);
      if (twod) {
        CHECK(hipMemcpy2DAsync(dev + c0, bs, src + c0, bs, n, k, hipMemcpyHostToDevice, sa));
      } else {
        for (int j = 0; j < k; ++j)
          CHECK(hipMemcpyAsync(dev + (size_t)j * bs + c0, src + (size_t)j * bs + c0, n,
                               hipMemcpyHostToDevice, sa));
      }
      CHECK(hipEventRecord(ev[c % 64], sa));
      CHECK(hipStreamWaitEvent(sb, ev[c % 64], 0));
      if (twod) {
        CHECK(hipMemcpy2DAsync(out + c0, bs, dev + (size_t)k * bs + c0, bs, n, m,
                               hipMemcpyDeviceToHost, sb));
      } else {
        for (int i = 0; i < m; ++i)
          CHECK(hipMemcpyAsync(out + (size_t)i * bs + c0, dev + (size_t)(k + i) * bs + c0, n,
                               hipMemcpyDeviceToHost, sb));
      }
    }
    CHECK(hipStreamSynchronize(sb));
    CHECK(hipStreamSynchronize(sa));
    if (r) reg(false);
  };

  if (poison) {
    // do pageable async copies of memory that was registered and
    // unregistered once read slower than before? (the same copies, timed
    // before and after one hipHostRegister / hipHostUnregister of the
    // buffers, and after it on a fresh buffer)
    auto med3 = [&](const char* what) {
      std::vector<double> v;
      for (int r = 0; r < 5; ++r) {
        const double t0 = now_ms();
        serial(false);
        v.push_back(now_ms() - t0);
      }
      std::sort(v.begin(), v.end());
      printf("{\"case\": \"serial pageable async, %s\", \"ms_med\": %.3f, \"ms_min\": %.3f}\n",
             what, v[2], v[0]);
    };
    med3("before any registration");
    reg(true);
    reg(false);
    med3("after one register + unregister of these buffers");
    uint8_t* src2 = static_cast<uint8_t*>(malloc((size_t)k * bs));
    uint8_t* out2 = static_cast<uint8_t*>(malloc((size_t)m * bs));
    memset(src2, 1, (size_t)k * bs);
    memset(out2, 2, (size_t)m * bs);
    std::swap(src, src2);
    std::swap(out, out2);
    med3("fresh buffers, never registered");
    return 0;
  }
  struct Case {
    std::string name;
    std::function<void()> fn;
  };
  std::vector<Case> cases = {{"serial", [&] { serial(false); }},
                             {"serial-reg", [&] { serial(true); }}};
  for (int C : {1, 2}) {
    cases.push_back({"chunk1d-reg-" + std::to_string(C), [&, C] { chunked(C, true, false); }});
  }
  for (int C : {4, 8, 16}) {
    cases.push_back({"chunk2d-" + std::to_string(C), [&, C] { chunked(C, false, true); }});
    cases.push_back({"chunk2d-reg-" + std::to_string(C), [&, C] { chunked(C, true, true); }});
    cases.push_back({"chunk1d-reg-" + std::to_string(C), [&, C] { chunked(C, true, false); }});
  }
  std::vector<std::vector<double>> t(cases.size());
  for (int round = 0; round < reps + 1; ++round) {
    for (size_t i = 0; i < cases.size(); ++i) {
      const double t0 = now_ms();
      cases[i].fn();
      const double dt = now_ms() - t0;
      if (round > 0) t[i].push_back(dt);  // round 0: warm-up
    }
  }
  // the register / unregister costs alone
  std::vector<double> tr, tu;
  for (int r = 0; r < reps; ++r) {
    double t0 = now_ms();
    reg(true);
    double t1 = now_ms();
    reg(false);
    tr.push_back(t1 - t0);
    tu.push_back(now_ms() - t1);
  }
  std::sort(tr.begin(), tr.end());
  std::sort(tu.begin(), tu.end());
  printf("{\"case\": \"register+unregister alone\", \"register_ms\": %.3f, \"unregister_ms\": %.3f}\n",
         tr[tr.size() / 2], tu[tu.size() / 2]);
  const double link = (double)(k + m) * bs;
  for (size_t i = 0; i < cases.size(); ++i) {
    std::sort(t[i].begin(), t[i].end());
    const double ms = t[i][t[i].size() / 2];
    printf("{\"case\": \"%s\", \"ms_med\": %.3f, \"ms_min\": %.3f, \"payload_GiBps\": %.1f, "
           "\"link_GBps\": %.1f}\n",
           cases[i].name.c_str(), ms, t[i][0], (double)size / ms * 1e3 / (1u << 30),
           link / ms / 1e6);
  }
  CHECK(hipFree(dev));
  free(src);
  free(out);
  return 0;
}
