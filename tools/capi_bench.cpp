// capi_bench.cpp — measurement only: the host-memory C ABI (the NIF's entry
// points) driven from plain C++ threads, with no Python and no torch in the
// process, i.e. on the system HIP runtime (/opt/rocm) the library resolves
// when an Erlang VM loads the NIF.  (Python tools run the engine on the HIP
// runtime the torch wheel bundles, a different build; the two read the same
// on these benchmarks, profiles/r04_s8_capi_*.log.)
//
//   g++ -O2 -std=c++17 -pthread -o tools/capi_bench tools/capi_bench.cpp -ldl
//   tools/capi_bench <libleoec*.so> ref      [K=V,...]   the reference's eunit
//                                                        encode benchmark (one
//                                                        100 MiB zero object per
//                                                        class; cold + warm calls)
//   tools/capi_bench <libleoec*.so> callers  [K=V,...]   1 MiB RS(10,4,8) encode /
//                                                        decode from 1, 8, 32 threads
//   tools/capi_bench <libleoec*.so> threads  [K=V,...]   first calls of new threads
//                                                        after gf_init on the main one
//   tools/capi_bench <libleoec*.so> few      [K=V,...]   callers() from 1, 2, 4, 8 threads
//   tools/capi_bench <libleoec*.so> mid      [K=V,...]   callers() from 4, 8, 16, 32 threads
//   tools/capi_bench <libleoec*.so> sizes    [K=V,...]   callers() at 16 KiB - 4 MiB
//                                                        objects, 8 and 32 threads
//   tools/capi_bench <libleoec*.so> many     [K=V,...]   callers() from 32 - 96 threads
//   tools/capi_bench <libleoec*.so> trace32  [K=V,...]   callers() from 32 threads,
//                                                        encode then decode (copy trace)
// K=V: measurement-build knobs (leoec_measure_set_knob), applied after load.
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

using GfInit = int (*)();
using Layout = int (*)(int, int, int, int, uint64_t, uint64_t*, int*);
using Encode = int (*)(int, int, int, int, const uint8_t*, uint64_t, uint8_t*, uint64_t);
using Decode = int (*)(int, int, int, int, const uint8_t* const*, const int*, int, uint64_t,
                       uint64_t, uint8_t*);
using SetKnob = int (*)(const char*, const char*);

using Stats = void (*)(double*);

GfInit gf_init;
Stats hostq_stats;  // measurement build only (nullptr otherwise)
Layout layout;
Encode encode;
Decode decode;

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

void* sym(void* h, const char* name) {
  void* p = dlsym(h, name);
  if (!p) {
    fprintf(stderr, "missing symbol %s\n", name);
    exit(2);
  }
  return p;
}

// bench_encode_test (test/leo_erasure_tests.erl:207-212, 304-336): one encode
// of a 100 MiB zero binary per class, rate = 100 / seconds.
void ref_bench(int reps) {
  struct Cls {
    const char* name;
    int id, k, m, w;
  };
  const Cls classes[] = {{"vandrs", 2, 10, 4, 8}, {"cauchyrs", 1, 10, 4, 10},
                         {"liberation", 3, 10, 2, 11}, {"isars", 4, 10, 4, 8}};
  const uint64_t size = 100ull << 20;
  for (const Cls& c : classes) {
    uint64_t bs;
    int filled;
    if (layout(c.id, c.k, c.m, c.w, size, &bs, &filled)) exit(3);
    const uint64_t outn = (uint64_t)(c.k + c.m - filled) * bs;
    std::vector<uint8_t> src(size, 0), out(outn, 0xA5);  // written: a fresh binary
    auto call = [&] {
      const double t0 = now_s();
      const int rc = encode(c.id, c.k, c.m, c.w, src.data(), size, out.data(), outn);
      const double dt = now_s() - t0;
      if (rc) {
        fprintf(stderr, "%s: rc %d\n", c.name, rc);
        exit(4);
      }
      for (uint64_t i = 0; i < outn; i += 4093)
        if (out[i]) {
          fprintf(stderr, "%s: non-zero output\n", c.name);
          exit(5);
        }
      return dt;
    };
    const double cold = call();
    std::vector<double> warm;
    for (int r = 0; r < reps; ++r) {
      std::fill(out.begin(), out.end(), 0xA5);
      warm.push_back(call());
    }
    std::sort(warm.begin(), warm.end());
    const double med = warm[warm.size() / 2];
    printf("{\"bench\": \"reference bench_encode_test, C ABI leoec_encode, 1 caller, system HIP "
           "runtime\", \"class\": \"%s\", \"params\": [%d, %d, %d], \"cold_ms\": %.2f, "
           "\"cold_MiBps\": %.1f, \"warm_ms\": %.2f, \"warm_MiBps\": %.1f, \"warm_min_ms\": %.2f}\n",
           c.name, c.k, c.m, c.w, cold * 1e3, 100.0 / cold, med * 1e3, 100.0 / med,
           warm[0] * 1e3);
    fflush(stdout);
  }
}

// tools/e2e_bench.py's callers(): T threads calling back to back, RS(10,4,8)
// objects of `size` bytes (1 MiB: the bench's), 3 trials of 0.4 s after a
// warm-up trial, median.
void callers(int T, bool dec, uint64_t size = 1ull << 20) {
  const int K = 10, M = 4, W = 8;
  uint64_t bs;
  int filled;
  if (layout(2, K, M, W, size, &bs, &filled)) exit(3);
  const uint64_t outn = (uint64_t)(K + M - filled) * bs;
  std::vector<std::vector<uint8_t>> srcs(T), outs(T), decs(T);
  std::vector<std::vector<const uint8_t*>> ptrs(T);
  std::vector<int> ids;
  for (int i = 4; i < K + M; ++i) ids.push_back(i);
  for (int t = 0; t < T; ++t) {
    std::mt19937_64 g(t + 1);
    srcs[t].resize(size);
    for (auto& b : srcs[t]) b = (uint8_t)g();
    outs[t].resize(outn);
    decs[t].resize(size);
    if (encode(2, K, M, W, srcs[t].data(), size, outs[t].data(), outn)) exit(4);
    for (int i : ids)
      ptrs[t].push_back(i < filled ? srcs[t].data() + (uint64_t)i * bs
                                   : outs[t].data() + (uint64_t)(i - filled) * bs);
  }
  std::atomic<int> errs{0};
  double calls_per_s = 0;
  auto call = [&](int t) {
    const int rc = dec ? decode(2, K, M, W, ptrs[t].data(), ids.data(), (int)ids.size(), bs, size,
                                decs[t].data())
                       : encode(2, K, M, W, srcs[t].data(), size, outs[t].data(), outn);
    if (rc) errs++;
  };
  auto trial = [&](double per) {
    std::vector<long> counts(T, 0);
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    double end = 0;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        call(t);  // warm this thread outside the timed region
        ready++;
        while (!go.load()) std::this_thread::yield();
        long n = 0;
        while (now_s() < end) {
          call(t);
          ++n;
        }
        counts[t] = n;
      });
    while (ready.load() < T) std::this_thread::yield();
    const double t0 = now_s();
    end = t0 + per;
    go = true;
    for (auto& x : th) x.join();
    const double dt = now_s() - t0;
    long n = 0;
    for (long c : counts) n += c;
    calls_per_s = n / dt;
    return n * (double)size / dt / (double)(1ull << 30);
  };
  trial(0.4);
  double st[14] = {};
  if (hostq_stats) hostq_stats(st);  // reset
  std::vector<double> r = {trial(0.4), trial(0.4), trial(0.4)};
  if (hostq_stats) hostq_stats(st);
  std::sort(r.begin(), r.end());
  if (dec)
    for (int t = 0; t < T; ++t)
      if (decs[t] != srcs[t]) {
        fprintf(stderr, "decode mismatch\n");
        exit(6);
      }
  std::string q;
  if (hostq_stats && st[0] > 0) {
    // per batch: jobs, then the timeline (us): worker waiting for fills,
    // issue, completer waiting on the GPU, open -> close, done -> free;
    // per job: caller waiting for DONE, waiting to reserve
    char b[512];
    snprintf(b, sizeof b,
             ", \"queue\": {\"batches\": %.0f, \"jobs_per_batch\": %.2f, \"launches_per_batch\": %.2f, "
             "\"fill_wait_us\": %.1f, \"issue_us\": %.1f, \"gpu_wait_us\": %.1f, "
             "\"open_to_close_us\": %.1f, \"done_to_free_us\": %.1f, \"caller_wait_us_per_job\": %.1f, "
             "\"reserve_wait_us_per_job\": %.1f}",
             st[0], st[1] / st[0], st[2] / st[0], st[3] / st[0], st[4] / st[0], st[5] / st[0],
             st[6] / st[0], st[7] / st[0], st[8] / std::max(st[1], 1.0), st[9] / std::max(st[1], 1.0));
    q = b;
  }
  printf("{\"path\": \"C ABI leoec_%s, %llu B objects, %d caller threads, system HIP runtime\", "
         "\"GiBps\": %.2f, \"GiBps_min_max\": [%.2f, %.2f], \"calls_per_s_last_trial\": %.0f, "
         "\"errors\": %d%s}\n",
         dec ? "decode" : "encode", (unsigned long long)size, T, r[1], r[0], r[2], calls_per_s,
         errs.load(), q.c_str());
  fflush(stdout);
}

// A VM calls gf_init on one thread and encodes on others (dirty
// schedulers): the first call of each new thread, 1 MiB and 100 MiB.
void new_threads() {
  for (uint64_t size : {1ull << 20, 100ull << 20}) {
    uint64_t bs;
    int filled;
    if (layout(2, 10, 4, 8, size, &bs, &filled)) exit(3);
    const uint64_t outn = (uint64_t)(14 - filled) * bs;
    std::vector<uint8_t> src(size, 0), out(outn, 0);
    for (int i = 0; i < 3; ++i) {
      double first = 0, second = 0;
      std::thread t([&] {
        double t0 = now_s();
        if (encode(2, 10, 4, 8, src.data(), size, out.data(), outn)) exit(4);
        first = now_s() - t0;
        t0 = now_s();
        if (encode(2, 10, 4, 8, src.data(), size, out.data(), outn)) exit(4);
        second = now_s() - t0;
      });
      t.join();
      printf("{\"bench\": \"first calls of a new thread after gf_init on another\", \"size\": %llu, "
             "\"thread\": %d, \"first_ms\": %.3f, \"second_ms\": %.3f}\n",
             (unsigned long long)size, i, first * 1e3, second * 1e3);
      fflush(stdout);
    }
  }
}

// One thread, back-to-back 1 MiB RS(10,4,8) encodes (a short target for a
// kernel / API trace of the lone-caller path): `n` calls, mean per call.
void lone(int n) {
  const uint64_t size = 1ull << 20;
  uint64_t bs;
  int filled;
  if (layout(2, 10, 4, 8, size, &bs, &filled)) exit(3);
  const uint64_t outn = (uint64_t)(14 - filled) * bs;
  std::vector<uint8_t> src(size, 7), out(outn, 0);
  for (int i = 0; i < 50; ++i)
    if (encode(2, 10, 4, 8, src.data(), size, out.data(), outn)) exit(4);
  const double t0 = now_s();
  for (int i = 0; i < n; ++i)
    if (encode(2, 10, 4, 8, src.data(), size, out.data(), outn)) exit(4);
  const double dt = now_s() - t0;
  printf("{\"bench\": \"lone caller, 1 MiB encodes back to back\", \"calls\": %d, "
         "\"us_per_call\": %.2f, \"GiBps\": %.2f}\n",
         n, dt / n * 1e6, n * (double)size / dt / (double)(1ull << 30));
  // decodes of data blocks 0-3 from blocks 4..13
  std::vector<int> ids;
  std::vector<const uint8_t*> ptrs;
  for (int i = 4; i < 14; ++i) {
    ids.push_back(i);
    ptrs.push_back(i < filled ? src.data() + (uint64_t)i * bs : out.data() + (uint64_t)(i - filled) * bs);
  }
  std::vector<uint8_t> dec(size);
  for (int i = 0; i < 50; ++i)
    if (decode(2, 10, 4, 8, ptrs.data(), ids.data(), 10, bs, size, dec.data())) exit(4);
  const double t1 = now_s();
  for (int i = 0; i < n; ++i)
    if (decode(2, 10, 4, 8, ptrs.data(), ids.data(), 10, bs, size, dec.data())) exit(4);
  const double dt2 = now_s() - t1;
  if (dec != src) exit(6);
  printf("{\"bench\": \"lone caller, 1 MiB decodes (lose 0-3) back to back\", \"calls\": %d, "
         "\"us_per_call\": %.2f, \"GiBps\": %.2f}\n",
         n, dt2 / n * 1e6, n * (double)size / dt2 / (double)(1ull << 30));
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <libleoec*.so> ref|callers [K=V,...]\n", argv[0]);
    return 2;
  }
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "%s\n", dlerror());
    return 2;
  }
  gf_init = (GfInit)sym(h, "leoec_gf_init");
  layout = (Layout)sym(h, "leoec_layout");
  encode = (Encode)sym(h, "leoec_encode");
  decode = (Decode)sym(h, "leoec_decode");
  hostq_stats = (Stats)dlsym(h, "leoec_measure_hostq_stats");
  if (argc > 3 && argv[3][0]) {
    auto set = (SetKnob)sym(h, "leoec_measure_set_knob");
    std::string kv = argv[3];
    size_t p = 0;
    while (p < kv.size()) {
      size_t q = kv.find(',', p);
      if (q == std::string::npos) q = kv.size();
      const std::string e = kv.substr(p, q - p);
      const size_t eq = e.find('=');
      if (eq != std::string::npos && set(e.substr(0, eq).c_str(), e.substr(eq + 1).c_str())) {
        fprintf(stderr, "knob %s refused\n", e.c_str());
        return 2;
      }
      p = q + 1;
    }
    printf("# knobs %s\n", argv[3]);
  }
  const double t0 = now_s();
  const int rc = gf_init();
  printf("{\"bench\": \"gf_init\", \"rc\": %d, \"ms\": %.2f}\n", rc, (now_s() - t0) * 1e3);
  if (rc) return 3;
  const std::string mode = argv[2];
  if (mode == "ref") {
    ref_bench(5);
  } else if (mode == "threads") {
    new_threads();
  } else if (mode == "lone") {
    lone(2000);
  } else if (mode == "few") {
    // the reference's basho_bench concurrency (test/basho_bench_leo_erasure_
    // rs_10_4_8_1M_w_t1 / _t4.config: {concurrent, 1 | 4}) and 2
    for (bool dec : {false, true})
      for (int T : {1, 2, 4, 8}) callers(T, dec);
  } else if (mode == "mid") {
    // where the per-thread path hands over to the batching queue
    for (bool dec : {false, true})
      for (int T : {4, 8, 16, 32}) callers(T, dec);
  } else if (mode == "c32") {
    // 32 callers, encode then decode (the bench host leg's concurrency; A/B)
    for (bool dec : {false, true}) callers(32, dec);
  } else if (mode == "many") {
    // 32, 48, 64, 96 callers: whether more callers' packing overlaps the
    // link's idle gaps (round 6: at 32 the next batch's last packs end after
    // the previous batch's H2D, tools/copy_gaps.py)
    for (bool dec : {false, true})
      for (int T : {32, 48, 64, 96}) callers(T, dec);
  } else if (mode == "trace32") {
    // the bench host leg's shape for a copy trace (rocprofv3 --kernel-trace
    // --memory-copy-trace; tools/copy_gaps.py): 32 callers, encode then decode
    for (bool dec : {false, true}) callers(32, dec);
  } else if (mode == "small") {
    // 16 KiB objects, 32 callers, encode (the queue's per-call cost)
    callers(32, false, 16ull << 10);
    callers(32, false, 64ull << 10);
  } else if (mode == "sizes") {
    // objects from 16 KiB to 4 MiB: the host path's per-call cost against
    // its bytes (RS(10,4,8); 8 and 32 callers)
    for (uint64_t size : {16ull << 10, 64ull << 10, 256ull << 10, 1ull << 20, 4ull << 20})
      for (bool dec : {false, true})
        for (int T : {8, 32}) callers(T, dec, size);
  } else {
    for (bool dec : {false, true})
      for (int T : {1, 8, 32}) callers(T, dec);
  }
  return 0;
}
