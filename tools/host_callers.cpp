// host_callers.cpp — measurement only (bench.py's host leg): caller threads
// in native code for the C ABI's host-memory entry points, as an Erlang VM's
// dirty schedulers call a NIF — no interpreter between the threads and
// leoec_encode / leoec_decode (Python threads through ctypes serialise on the
// interpreter lock around every call: 41-42 GiB/s against 46 from C++
// callers at 32 threads, round 5-6 bench lines against tools/capi_bench).
//
// The caller passes the entry points' addresses (from the library it
// loaded) and every thread's buffers; each thread makes one call outside the
// clock, waits at a barrier, then calls back to back until `seconds` pass.
//   g++ -O2 -std=c++17 -shared -fPIC -pthread -o tools/libhost_callers.so tools/host_callers.cpp
#include <atomic>
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

using Encode = int (*)(int, int, int, int, const uint8_t*, uint64_t, uint8_t*, uint64_t);
using Decode = int (*)(int, int, int, int, const uint8_t* const*, const int*, int, uint64_t,
                       uint64_t, uint8_t*);

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// op 0: encode(coding, k, m, w, srcs[t], size, outs[t], out_bytes);
// op 1: decode(coding, k, m, w, ptrs[t * nids ..], ids, nids, bs, size, outs[t]).
// counts[t] = calls of thread t in the timed window; *elapsed = the window
// (seconds).  Returns the number of calls that failed (0: every call ok).
extern "C" __attribute__((visibility("default"))) long host_callers_run(
    void* fn, int op, int nthreads, double seconds, int coding, int k, int m, int w,
    const uint8_t* const* srcs, uint8_t* const* outs, uint64_t size, uint64_t out_bytes,
    const uint8_t* const* ptrs, const int* ids, int nids, uint64_t bs, long* counts,
    double* elapsed) {
  std::atomic<long> errors{0};
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  double end = 0;
  auto call = [&](int t) {
    if (op == 0)
      return reinterpret_cast<Encode>(fn)(coding, k, m, w, srcs[t], size, outs[t], out_bytes);
    return reinterpret_cast<Decode>(fn)(coding, k, m, w, ptrs + (size_t)t * nids, ids, nids, bs,
                                        size, outs[t]);
  };
  std::vector<std::thread> th;
  th.reserve(nthreads);
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&, t] {
      if (call(t) != 0) errors++;  // this thread's first call, outside the clock
      ready++;
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      long c = 0;
      while (now_s() < end) {
        if (call(t) != 0) errors++;
        ++c;
      }
      counts[t] = c;
    });
  while (ready.load() < nthreads) std::this_thread::yield();
  const double t0 = now_s();
  end = t0 + seconds;
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  *elapsed = now_s() - t0;
  return errors.load();
}
