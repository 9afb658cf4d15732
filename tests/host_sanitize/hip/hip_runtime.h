// A CPU stand-in for the HIP runtime, TEST INFRASTRUCTURE ONLY: it lets the
// engine's host C++ (engine.cpp, hostq.cpp, capi.cpp, codes.cpp, knobs.cpp)
// build with g++ under AddressSanitizer / UndefinedBehaviorSanitizer and
// ThreadSanitizer (tests/host_sanitize/Makefile, tests/test_host_sanitize.py).
// It is never part of a product build: the engine's own builds include the
// real <hip/hip_runtime.h> from /opt/rocm.
//
// What it models, so the sanitizers see the engine's real orderings:
//   * streams are in-order queues, each drained by its own thread, with a
//     random delay of up to ~50 us before every operation (widens race
//     windows); events complete when the operations enqueued before their
//     record have run; hipStreamSynchronize / hipEventSynchronize /
//     hipEventQuery wait on or poll exactly that;
//   * memory: hipMalloc / hipHostMalloc are plain heap blocks (ASan sees
//     every out-of-bounds "device" access), a mapped host block's device
//     pointer is itself; copies from or to memory that is not from
//     hipHostMalloc (pageable) complete before hipMemcpyAsync returns, as
//     the HIP runtime's staged pageable copies do, pinned copies are
//     asynchronous;
//   * two "gfx950" devices with a per-thread current device.
// Kernels are the engine's launch() entry points, implemented on the CPU in
// fake_kernels.cpp and run on the stream's thread.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <random>
#include <thread>

typedef enum hipError_t {
  hipSuccess = 0,
  hipErrorInvalidValue = 1,
  hipErrorOutOfMemory = 2,
  hipErrorInvalidDevice = 101,
  hipErrorNotReady = 600,
  hipErrorHostMemoryAlreadyRegistered = 712,
  hipErrorHostMemoryNotRegistered = 713,
} hipError_t;

typedef enum hipMemcpyKind {
  hipMemcpyHostToHost = 0,
  hipMemcpyHostToDevice = 1,
  hipMemcpyDeviceToHost = 2,
  hipMemcpyDeviceToDevice = 3,
} hipMemcpyKind;

#define hipStreamNonBlocking 0x01
#define hipEventDefault 0x0
#define hipEventBlockingSync 0x1
#define hipEventDisableTiming 0x2
#define hipHostMallocDefault 0x0
#define hipHostMallocMapped 0x2
#define hipHostRegisterDefault 0x0
#define hipHostRegisterPortable 0x1
#define hipHostRegisterMapped 0x2

struct hipDeviceProp_t {
  char name[256];
  char gcnArchName[256];
};

namespace fakehip {

constexpr int kDevices = 2;

struct Stream {
  int device = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  uint64_t enq = 0, done = 0;
  bool stop = false;
  std::thread th;

  explicit Stream(int dev) : device(dev) {
    th = std::thread([this] { run(); });
  }
  ~Stream() {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    th.join();
  }
  void run() {
    std::mt19937 rng((unsigned)(uintptr_t)this);
    std::unique_lock<std::mutex> l(mu);
    for (;;) {
      cv.wait(l, [this] { return stop || !q.empty(); });
      if (q.empty()) return;
      std::function<void()> op = std::move(q.front());
      q.pop_front();
      l.unlock();
      std::this_thread::sleep_for(std::chrono::microseconds(rng() % 50));
      op();
      l.lock();
      ++done;
      cv.notify_all();
    }
  }
  uint64_t push(std::function<void()> op) {
    std::lock_guard<std::mutex> l(mu);
    q.push_back(std::move(op));
    const uint64_t t = ++enq;
    cv.notify_all();
    return t;
  }
  uint64_t ticket() {
    std::lock_guard<std::mutex> l(mu);
    return enq;
  }
  void wait(uint64_t t) {
    std::unique_lock<std::mutex> l(mu);
    cv.wait(l, [this, t] { return done >= t; });
  }
  bool reached(uint64_t t) {
    std::lock_guard<std::mutex> l(mu);
    return done >= t;
  }
};

struct Event {
  std::mutex mu;
  Stream* s = nullptr;
  uint64_t t = 0;
};

inline int& current_device() {
  static thread_local int d = 0;
  return d;
}

// The legacy null stream of each device (the engine always passes its own).
inline Stream* null_stream() {
  static Stream* s[kDevices] = {new Stream(0), new Stream(1)};
  return s[current_device()];
}

struct Pinned {
  std::mutex mu;
  std::map<uintptr_t, size_t> blocks;  // base -> bytes (hipHostMalloc and hipHostRegister)
  std::map<uintptr_t, int> registered; // hipHostRegister base -> copies in flight
  long n_registered = 0, n_refused = 0;  // hipHostRegister calls that pinned / were refused
  bool contains(const void* p, size_t n) {
    std::lock_guard<std::mutex> l(mu);
    return base_of(p, n) != 0;
  }
  uintptr_t base_of(const void* p, size_t n) {  // mu held
    const uintptr_t a = (uintptr_t)p;
    auto it = blocks.upper_bound(a);
    if (it == blocks.begin()) return 0;
    --it;
    return a >= it->first && a + n <= it->first + it->second ? it->first : 0;
  }
  // a copy from / to registered memory starts (true) or ends: counted, so
  // unregistering memory under a copy in flight is caught
  void track(const void* p, size_t n, int d) {
    std::lock_guard<std::mutex> l(mu);
    const uintptr_t b = base_of(p, n);
    auto it = registered.find(b);
    if (it != registered.end()) it->second += d;
  }
};
inline Pinned& pinned() {
  static Pinned* p = new Pinned;
  return *p;
}

// Fault injection: the n-th hipEventCreateWithFlags of the calling thread
// from now on fails (0: none).  host_stress uses it to fail the second
// column chunk of a per-thread zero-copy call (engine.cpp zc_chunked).
inline int& fail_event_create_in() {
  static thread_local int n = 0;
  return n;
}
inline void fail_nth_event_create(int n) { fail_event_create_in() = n; }

// Thread teardown: set on a thread once the first of its thread_local
// destructors has started (tls_teardown.cpp re-registers the marker after
// every thread_local destructor registration, so it runs before all of
// them).  A HIP call from then on is what made rocprofv3 abort the bench's
// host leg (profiles/r05_s6_bench_prof_host_leg_abort.txt: the tool's own
// thread-local state may already be gone): every fake entry point aborts on it.
inline bool& tls_teardown() {
  static thread_local bool f = false;  // trivially destructible: no registration
  return f;
}
inline void live(const char* fn) {
  if (tls_teardown()) {
    std::fprintf(stderr, "fake hip: %s called during thread-local teardown\n", fn);
    std::abort();
  }
}

inline std::atomic<long>& live_allocs() {
  static std::atomic<long> n{0};
  return n;
}

}  // namespace fakehip

typedef fakehip::Stream* hipStream_t;
typedef fakehip::Event* hipEvent_t;

inline hipError_t hipGetDeviceCount(int* n) {
  fakehip::live("hipGetDeviceCount");
  *n = fakehip::kDevices;
  return hipSuccess;
}
inline hipError_t hipGetDeviceProperties(hipDeviceProp_t* p, int dev) {
  fakehip::live("hipGetDeviceProperties");
  if (dev < 0 || dev >= fakehip::kDevices) return hipErrorInvalidDevice;
  std::memset(p, 0, sizeof(*p));
  std::strcpy(p->name, "fake MI355X (host sanitizer harness)");
  std::strcpy(p->gcnArchName, "gfx950:sramecc+:xnack-");
  return hipSuccess;
}
inline hipError_t hipSetDevice(int dev) {
  fakehip::live("hipSetDevice");
  if (dev < 0 || dev >= fakehip::kDevices) return hipErrorInvalidDevice;
  fakehip::current_device() = dev;
  return hipSuccess;
}
inline hipError_t hipGetDevice(int* dev) {
  fakehip::live("hipGetDevice");
  *dev = fakehip::current_device();
  return hipSuccess;
}

inline hipError_t hipMalloc(void** p, size_t n) {
  fakehip::live("hipMalloc");
  *p = std::malloc(n ? n : 1);
  if (!*p) return hipErrorOutOfMemory;
  ++fakehip::live_allocs();
  return hipSuccess;
}
template <class T>
inline hipError_t hipMalloc(T** p, size_t n) {
  fakehip::live("hipMalloc");
  return hipMalloc(reinterpret_cast<void**>(p), n);
}
inline hipError_t hipFree(void* p) {
  fakehip::live("hipFree");
  if (p) --fakehip::live_allocs();
  std::free(p);
  return hipSuccess;
}
inline hipError_t hipHostMalloc(void** p, size_t n, unsigned) {
  fakehip::live("hipHostMalloc");
  *p = std::malloc(n ? n : 1);
  if (!*p) return hipErrorOutOfMemory;
  ++fakehip::live_allocs();
  std::lock_guard<std::mutex> l(fakehip::pinned().mu);
  fakehip::pinned().blocks[(uintptr_t)*p] = n;
  return hipSuccess;
}
inline hipError_t hipHostFree(void* p) {
  fakehip::live("hipHostFree");
  if (p) {
    --fakehip::live_allocs();
    std::lock_guard<std::mutex> l(fakehip::pinned().mu);
    fakehip::pinned().blocks.erase((uintptr_t)p);
  }
  std::free(p);
  return hipSuccess;
}
inline hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) {
  fakehip::live("hipHostGetDevicePointer");
  // only pinned memory (hipHostMalloc, hipHostRegister) has a device address
  if (!fakehip::pinned().contains(h, 1)) {
    *d = nullptr;
    return hipErrorInvalidValue;
  }
  *d = h;
  return hipSuccess;
}

inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {
  fakehip::live("hipStreamCreateWithFlags");
  *s = new fakehip::Stream(fakehip::current_device());
  return hipSuccess;
}
inline hipError_t hipStreamDestroy(hipStream_t s) {
  fakehip::live("hipStreamDestroy");
  delete s;
  return hipSuccess;
}
inline fakehip::Stream* fake_stream(hipStream_t s) { return s ? s : fakehip::null_stream(); }
inline hipError_t hipStreamSynchronize(hipStream_t s) {
  fakehip::live("hipStreamSynchronize");
  fakehip::Stream* st = fake_stream(s);
  st->wait(st->ticket());
  return hipSuccess;
}

inline hipError_t hipStreamQuery(hipStream_t s) {
  fakehip::live("hipStreamQuery");
  fakehip::Stream* st = fake_stream(s);
  return st->reached(st->ticket()) ? hipSuccess : hipErrorNotReady;
}

inline hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, hipMemcpyKind kind,
                                 hipStream_t s) {
  fakehip::live("hipMemcpyAsync");
  fakehip::Stream* st = fake_stream(s);
  const void* host = kind == hipMemcpyHostToDevice ? src : kind == hipMemcpyDeviceToHost ? dst
                                                                                          : nullptr;
  if (host) fakehip::pinned().track(host, n, +1);
  const uint64_t t = st->push([dst, src, n, host] {
    std::memcpy(dst, src, n);
    if (host) fakehip::pinned().track(host, n, -1);
  });
  // pageable host memory: the runtime's staged copy is done on return
  if (host && !fakehip::pinned().contains(host, n)) st->wait(t);
  return hipSuccess;
}

// Pins caller memory in place: copies to / from it become asynchronous like
// any pinned copy.  Overlapping an existing pinned block is refused, as the
// runtime refuses it; unregistering under a copy in flight aborts the test.
inline hipError_t hipHostRegister(void* p, size_t n, unsigned) {
  fakehip::live("hipHostRegister");
  fakehip::Pinned& pn = fakehip::pinned();
  std::lock_guard<std::mutex> l(pn.mu);
  const uintptr_t a = (uintptr_t)p;
  auto it = pn.blocks.upper_bound(a + n - 1);
  if (it != pn.blocks.begin()) {
    --it;
    if (it->first + it->second > a) {
      ++pn.n_refused;
      return hipErrorHostMemoryAlreadyRegistered;
    }
  }
  ++pn.n_registered;
  pn.blocks[a] = n;
  pn.registered[a] = 0;
  return hipSuccess;
}
inline hipError_t hipHostUnregister(void* p) {
  fakehip::live("hipHostUnregister");
  fakehip::Pinned& pn = fakehip::pinned();
  std::lock_guard<std::mutex> l(pn.mu);
  auto it = pn.registered.find((uintptr_t)p);
  if (it == pn.registered.end()) return hipErrorHostMemoryNotRegistered;
  if (it->second != 0) {
    std::fprintf(stderr, "fake hip: hipHostUnregister(%p) with %d copies in flight\n", p,
                 it->second);
    std::abort();
  }
  pn.registered.erase(it);
  pn.blocks.erase((uintptr_t)p);
  return hipSuccess;
}

inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  fakehip::live("hipEventCreateWithFlags");
  int& n = fakehip::fail_event_create_in();
  if (n > 0 && --n == 0) {
    *e = nullptr;
    return hipErrorOutOfMemory;
  }
  *e = new fakehip::Event;
  return hipSuccess;
}
inline hipError_t hipEventDestroy(hipEvent_t e) {
  fakehip::live("hipEventDestroy");
  delete e;
  return hipSuccess;
}
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
  fakehip::live("hipEventRecord");
  fakehip::Stream* st = fake_stream(s);
  std::lock_guard<std::mutex> l(e->mu);
  e->s = st;
  e->t = st->ticket();
  return hipSuccess;
}
inline hipError_t hipEventQuery(hipEvent_t e) {
  fakehip::live("hipEventQuery");
  fakehip::Stream* st;
  uint64_t t;
  {
    std::lock_guard<std::mutex> l(e->mu);
    st = e->s;
    t = e->t;
  }
  return !st || st->reached(t) ? hipSuccess : hipErrorNotReady;
}
inline hipError_t hipEventSynchronize(hipEvent_t e) {
  fakehip::live("hipEventSynchronize");
  fakehip::Stream* st;
  uint64_t t;
  {
    std::lock_guard<std::mutex> l(e->mu);
    st = e->s;
    t = e->t;
  }
  if (st) st->wait(t);
  return hipSuccess;
}

// Later work on s waits for what preceded e's record (on e's stream): the
// wait is an operation of s's own thread, as the device's barrier packet.
inline hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned) {
  fakehip::live("hipStreamWaitEvent");
  fakehip::Stream* on;
  uint64_t t;
  {
    std::lock_guard<std::mutex> l(e->mu);
    on = e->s;
    t = e->t;
  }
  if (!on) return hipSuccess;  // never recorded: nothing to wait for
  fake_stream(s)->push([on, t] { on->wait(t); });
  return hipSuccess;
}

inline const char* hipGetErrorString(hipError_t) { return "fake hip error"; }
inline hipError_t hipGetLastError() {
  fakehip::live("hipGetLastError");
  return hipSuccess;
}
