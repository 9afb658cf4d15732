// hostq.cpp — see hostq.hpp.
//
// Per device: kSlots batch slots, each a pinned input arena + pinned output
// arena + their device twins, a stream and its events, and two copy streams
// shared by the slots (every batch's H2D on one, every D2H on the other: the
// link's two directions overlap only when their copies are on separate
// streams, tools/duplex_probe.hip).  A slot moves
//   FREE -> OPEN (callers reserve space and copy their inputs in)
//        -> CLOSED (no more reservations; the worker waits for the copies)
//        -> INFLIGHT (H2D on the input-copy stream, launches on the slot's
//                     stream, D2H on the output-copy stream, chained by events)
//        -> DONE (callers copy their outputs out) -> FREE (last reader).
// The worker closes the open slot whenever fewer than Knobs::hostq_depth
// batches are on the GPU, so calls arriving while the GPU is busy pile into
// one batch, and a lone call is launched at once.  The completer thread waits for batches
// in launch order and wakes their callers.
#include "hostq.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

#include "../../include/leoec.h"
#include "host_copy.hpp"
#include "knobs.hpp"

namespace leoec {

namespace {

constexpr int kSlots = 5;
constexpr uint64_t kSlotBytes = (uint64_t)16 << 20;  // input arena (and output arena) per batch
constexpr size_t kMaxJobs = 256;
constexpr uint64_t kAlign = 256;
static_assert(kBatchMaxJobBytes <= kSlotBytes, "a batched job must fit one slot");

uint64_t align_up(uint64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

using Clock = std::chrono::steady_clock;
double us_since(Clock::time_point t) {
  return std::chrono::duration<double, std::micro>(Clock::now() - t).count();
}

#ifdef LEOEC_MEASURE
// Queue timeline counters (measurement build): leoec_measure_hostq_stats.
struct Stats {
  std::mutex mu;
  double v[14] = {};  // batches, jobs, launches, fill_wait_us, issue_us, gpu_wait_us,
                      // open_to_close_us, done_to_free_us, caller_wait_us, reserve_wait_us,
                      // max issue_us, h2d enqueue us, launches us, d2h enqueue us
} g_stats;
void stat_add(int i, double x) {
  std::lock_guard<std::mutex> l(g_stats.mu);
  g_stats.v[i] += x;
}
double g_lane_jobs[64] = {};  // jobs launched per lane (under g_stats.mu)
void stat_lane_jobs(int lane, double n) {
  std::lock_guard<std::mutex> l(g_stats.mu);
  if (lane >= 0 && lane < 64) g_lane_jobs[lane] += n;
}
#else
inline void stat_add(int, double) {}
inline void stat_lane_jobs(int, double) {}
#endif

enum class St { kFree, kOpen, kClosed, kInflight, kDone };

struct Slot {
  St state = St::kFree;
  bool ready = false;  // buffers, stream and event exist
  uint8_t* h_in = nullptr;
  uint8_t* h_out = nullptr;
  uint8_t* d_in = nullptr;
  uint8_t* d_out = nullptr;
  uint8_t* z_in = nullptr;   // device addresses of h_in / h_out (zero-copy batches)
  uint8_t* z_out = nullptr;
  hipStream_t stream = nullptr;  // the slot's launches
  hipStream_t up = nullptr;      // the queue's input-copy stream (every slot's H2D)
  hipStream_t down = nullptr;    // the queue's output-copy stream (every slot's D2H)
  hipEvent_t ev = nullptr;
  hipEvent_t ev_blk = nullptr;  // the same, created hipEventBlockingSync (Knobs::hostq_sync = 2)
  hipEvent_t ev_done = nullptr; // the one recorded for this batch (ev or ev_blk)
  hipEvent_t ev_h2d = nullptr;  // after the input copy: the H2D engine is free for the next batch
  hipEvent_t ev_k = nullptr;    // after the launches: the output copy may start
  uint64_t used_in = 0, used_out = 0;
  std::vector<const HostJob*> jobs;
  std::vector<uint64_t> in_off, out_off;
  std::vector<int> job_rc;  // per job: its launch's status
  int lane = -1;
  int reserved = 0, filled = 0, readers = 0;
  int status = LEOEC_OK;    // the batch's copies and event: fails every job
  Clock::time_point opened, done;
  std::condition_variable cv_done;  // this batch's callers (Knobs::hostq_wake = 1)
};

struct Queue {
  int device = -1;
  hipStream_t up = nullptr, down = nullptr;  // the copy streams (Slot::up / down)
  std::mutex mu;
  std::condition_variable cv_worker;    // work for the worker (jobs, fills, GPU room)
  std::condition_variable cv_complete;  // work for the completer
  std::condition_variable cv_free;      // a slot became FREE
  std::condition_variable cv_done;      // a slot became DONE
  Slot slots[kSlots];
  Slot* open = nullptr;
  std::deque<Slot*> closed;    // closed by a caller because it was full
  std::atomic<int> nclosed{0}; // closed.size(), read without the lock (wait_h2d_or_closed)
  std::deque<Slot*> inflight;  // launch order
  Slot* last = nullptr;        // most recently launched
  int direct = 0;              // calls on their per-thread path (HostqTicket)
  int free_waiters = 0;        // callers waiting on cv_free
  int done_waiters = 0;        // callers waiting on cv_done (Knobs::hostq_wake = 0)
};

// Wait for `ev` without holding the queue lock: (Knobs::hostq_sync = 1) a
// hipEventQuery poll with yields, else hipEventSynchronize (= 2: on an event
// created hipEventBlockingSync, which sleeps instead of spinning).
hipError_t wait_event(hipEvent_t ev) {
  if (knobs().hostq_sync == 1) {
    for (;;) {
      const hipError_t e = hipEventQuery(ev);
      if (e != hipErrorNotReady) return e;
      std::this_thread::yield();
    }
  }
  return hipEventSynchronize(ev);
}

// The worker's wait for the previous batch's input copy (Knobs::hostq_close =
// 1), cut short when a caller hands over a complete batch meanwhile (it can
// be issued at once: its H2D queues behind the running one).  True when the
// copy is done.
bool wait_h2d_or_closed(hipEvent_t ev, const Queue* q) {
  if (knobs().hostq_sync != 1) {
    (void)wait_event(ev);  // (a failed copy is the batch's status: the completer reports it)
    return true;
  }
  for (;;) {
    if (hipEventQuery(ev) != hipErrorNotReady) return true;
    if (q->nclosed.load(std::memory_order_acquire) > 0) return false;
    std::this_thread::yield();
  }
}

int slot_alloc(Slot* s) {
  if (hipHostMalloc((void**)&s->h_in, kSlotBytes, hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc((void**)&s->h_out, kSlotBytes, hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&s->z_in, s->h_in, 0) != hipSuccess ||
      hipHostGetDevicePointer((void**)&s->z_out, s->h_out, 0) != hipSuccess ||
      hipMalloc((void**)&s->d_in, kSlotBytes) != hipSuccess ||
      hipMalloc((void**)&s->d_out, kSlotBytes) != hipSuccess ||
      hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_blk, hipEventDisableTiming | hipEventBlockingSync) !=
          hipSuccess ||
      hipEventCreateWithFlags(&s->ev_h2d, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_k, hipEventDisableTiming) != hipSuccess) {
    if (s->h_in) (void)hipHostFree(s->h_in);
    if (s->h_out) (void)hipHostFree(s->h_out);
    if (s->d_in) (void)hipFree(s->d_in);
    if (s->d_out) (void)hipFree(s->d_out);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    s->h_in = s->h_out = s->d_in = s->d_out = nullptr;
    s->stream = nullptr;
    return LEOEC_E_NOMEM;
  }
  s->ready = true;
  return LEOEC_OK;
}

bool same_map(const HostJob& a, const HostJob& b) {
  return (a.plan == b.plan ||
          (a.plan->code == b.plan->code && a.plan->surv == b.plan->surv &&
           a.plan->want == b.plan->want && a.plan->kind == b.plan->kind)) &&
         a.bs == b.bs && a.in_blk == b.in_blk && a.out_blk == b.out_blk &&
         a.out_valid == b.out_valid && a.in_bytes == b.in_bytes && a.out_bytes == b.out_bytes &&
         a.in_valid == b.in_valid;
}

// Enqueue one batch: ONE H2D of the input arena, one launch per run of
// consecutive identical maps (their regions are uniformly strided: they were
// reserved back to back with the same sizes), ONE D2H of the output arena.
// The copies go on the queue's two copy streams (Knobs::hostq_streams = 1,
// shipped), the launches on the slot's stream after the H2D's event, the
// D2H after the launches' event: batch b's D2H then runs beside batch b+1's
// H2D on the full-duplex link.  (hostq_streams = 0: all three on the slot's
// stream, the round-2..5 form, whose copies of neighbouring batches did not
// overlap on the link: profiles/r05_s19_duplex_queue.log.)
// Plans were built by the callers, so a launch can fail only for its own
// jobs (s->job_rc); the other runs are still launched.  The event is
// recorded whatever happened, so the completer always waits for the work
// that was enqueued before the slot can be reused.  Returns the status that
// fails every job (the copies, the event).
int launch_slot(Slot* s) {
  Clock::time_point t = Clock::now();
  // Knobs::hostq_zc (measurement): the kernels read the pinned input arena
  // and write the pinned output arena over PCIe, no DMA copy either way
  const bool zc = knobs().hostq_zc != 0;
  uint8_t* din = zc ? s->z_in : s->d_in;
  uint8_t* dout = zc ? s->z_out : s->d_out;
  // (small batches stay on the slot's stream: Knobs::hostq_split_kib)
  const bool split = !zc && knobs().hostq_streams == 1 && s->up && s->down &&
                     s->used_in >= ((uint64_t)knobs().hostq_split_kib << 10);
  hipStream_t cin = split ? s->up : s->stream;     // the input copy's stream
  hipStream_t cout = split ? s->down : s->stream;  // the output copy's stream
  int rc = zc ? LEOEC_OK
              : hipMemcpyAsync(s->d_in, s->h_in, s->used_in, hipMemcpyHostToDevice, cin) ==
                        hipSuccess
                    ? LEOEC_OK
                    : LEOEC_E_HIP;
  if (rc == LEOEC_OK && !zc && hipEventRecord(s->ev_h2d, cin) != hipSuccess) rc = LEOEC_E_HIP;
  if (rc == LEOEC_OK && split && hipStreamWaitEvent(s->stream, s->ev_h2d, 0) != hipSuccess)
    rc = LEOEC_E_HIP;
  stat_add(11, us_since(t));
  t = Clock::now();
  const size_t n = s->jobs.size();
  for (size_t i = 0; rc == LEOEC_OK && i < n;) {
    const HostJob& J = *s->jobs[i];
    const uint64_t sin = align_up(J.in_bytes), sout = align_up(J.out_bytes);
    size_t j = i + 1;
    while (j < n && same_map(J, *s->jobs[j]) && s->in_off[j] == s->in_off[j - 1] + sin &&
           s->out_off[j] == s->out_off[j - 1] + sout)
      ++j;
    const int k = J.plan->code->k, r = (int)J.plan->want.size();
    std::vector<Shard> in(k), out(r);
    for (int b = 0; b < k; ++b)
      in[b] = Shard{din + s->in_off[i] + (uint64_t)b * J.in_blk, sin, J.in_valid[b]};
    for (int o = 0; o < r; ++o)
      out[o] = Shard{dout + s->out_off[i] + (uint64_t)o * J.out_blk, sout, J.out_valid};
    int run_rc;
#ifdef LEOEC_MEASURE
    // fault injection (LEOEC_HOSTQ_FAIL_BS): this run's launch "fails"
    if (knobs().hostq_fail_bs > 0 && J.bs == (uint64_t)knobs().hostq_fail_bs)
      run_rc = LEOEC_E_HIP;
    else
#endif
      run_rc = run_plan(*J.plan, in, out, J.bs, (uint64_t)(j - i), s->stream);
    stat_lane_jobs(s->lane, (double)(j - i));
    for (size_t x = i; x < j; ++x) s->job_rc[x] = run_rc;
    stat_add(2, 1);
    i = j;
  }
  stat_add(12, us_since(t));
  t = Clock::now();
  if (rc == LEOEC_OK && zc && hipEventRecord(s->ev_h2d, s->stream) != hipSuccess)
    rc = LEOEC_E_HIP;  // (zero-copy: the inputs are consumed when the launches end)
  if (rc == LEOEC_OK && split &&
      (hipEventRecord(s->ev_k, s->stream) != hipSuccess ||
       hipStreamWaitEvent(cout, s->ev_k, 0) != hipSuccess))
    rc = LEOEC_E_HIP;
  if (rc == LEOEC_OK && !zc &&
      hipMemcpyAsync(s->h_out, s->d_out, s->used_out, hipMemcpyDeviceToHost, cout) != hipSuccess)
    rc = LEOEC_E_HIP;
  stat_add(13, us_since(t));
  s->ev_done = knobs().hostq_sync == 2 ? s->ev_blk : s->ev;
  hipStream_t last = cout;
  if (split && rc != LEOEC_OK) {
    // a failure part-way: drain whatever this batch enqueued on the three
    // streams, so the event below (on the slot's stream) follows all of it
    (void)hipStreamSynchronize(cin);
    (void)hipStreamSynchronize(s->stream);
    (void)hipStreamSynchronize(cout);
    last = s->stream;
  }
  if (hipEventRecord(s->ev_done, last) != hipSuccess) {
    (void)hipStreamSynchronize(last);  // no event to wait on: drain here
    if (split) (void)hipStreamSynchronize(s->stream);
    if (rc == LEOEC_OK) rc = LEOEC_E_HIP;
  }
  return rc;
}

void worker_main(Queue* q) {
  (void)hipSetDevice(q->device);
  std::unique_lock<std::mutex> lk(q->mu);
  for (;;) {
    const int depth = knobs().hostq_depth;
    q->cv_worker.wait(lk, [q, depth] {
      return (int)q->inflight.size() < depth &&
             (!q->closed.empty() || (q->open && q->open->reserved > 0));
    });
    // Knobs::hostq_close = 1: let the open batch grow until the previous
    // batch's input copy is done (the H2D engine has room for it)
    if (knobs().hostq_close == 1 && q->closed.empty() && q->last &&
        q->last->state == St::kInflight) {
      Slot* prev = q->last;
      lk.unlock();
      const bool copied = wait_h2d_or_closed(prev->ev_h2d, q);
      lk.lock();
      if (copied && q->last == prev) q->last = nullptr;
      continue;
    }
    Slot* s;
    if (!q->closed.empty()) {
      s = q->closed.front();
      q->closed.pop_front();
      q->nclosed.fetch_sub(1, std::memory_order_release);
    } else {
      s = q->open;
      // measurement knob: hold an idle-GPU batch open for a window
      const int win = knobs().batch_window_us;
      if (win > 0 && q->inflight.empty()) {
        const auto until = s->opened + std::chrono::microseconds(win);
        q->cv_worker.wait_until(lk, until, [q, s] { return q->open != s; });
        if (q->open != s) continue;  // a caller closed it (full): take it from `closed`
      }
      q->open = nullptr;
      s->state = St::kClosed;
    }
    stat_add(6, us_since(s->opened));
    const Clock::time_point tf = Clock::now();
    q->cv_worker.wait(lk, [s] { return s->filled == s->reserved; });
    stat_add(3, us_since(tf));
    stat_add(0, 1);
    stat_add(1, (double)s->jobs.size());
    s->state = St::kInflight;
    lk.unlock();
    const Clock::time_point tl = Clock::now();
    const int rc = launch_slot(s);
    const double iu = us_since(tl);
    stat_add(4, iu);
#ifdef LEOEC_MEASURE
    {
      std::lock_guard<std::mutex> l(g_stats.mu);
      if (iu > g_stats.v[10]) g_stats.v[10] = iu;
    }
#endif
    lk.lock();
    s->status = rc;
    q->inflight.push_back(s);
    q->last = s;
    q->cv_complete.notify_one();
  }
}

void completer_main(Queue* q) {
  (void)hipSetDevice(q->device);
  std::unique_lock<std::mutex> lk(q->mu);
  for (;;) {
    q->cv_complete.wait(lk, [q] { return !q->inflight.empty(); });
    Slot* s = q->inflight.front();
    lk.unlock();
    const Clock::time_point tw = Clock::now();
    const int rc = wait_event(s->ev_done) == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
    stat_add(5, us_since(tw));
    lk.lock();
    s->done = Clock::now();
    q->inflight.pop_front();
    if (q->last == s) q->last = nullptr;
    if (s->status == LEOEC_OK) s->status = rc;
    s->state = St::kDone;
    s->cv_done.notify_all();  // this batch's callers
    if (q->done_waiters > 0) q->cv_done.notify_all();  // (round-4 form: every caller)
    q->cv_worker.notify_one();
  }
}

// Dispatcher lanes: lane i runs on host_devices()[i % ndev], one lane per
// gfx950 device.  By default a host-memory call runs on the lane of the
// caller's current device (the reference NIF's contract: the library uses
// what the process was given, and one process per GPU stays on its GPU);
// leoec_host_spread() opts in to spreading calls over a set of devices, each
// call going to the lane with the fewest calls in progress.  The measurement
// knob LEOEC_HOSTQ_LANES maps more lanes onto fewer devices and spreads over
// all of them (the dispatcher's test on a one-GPU box).  Each lane has a
// queue, created on first use; its two threads live for the process (they
// hold no GPU work when idle, and a process exits with them parked on their
// condition variables; libleoec.so is linked -z nodelete so their code is
// never unmapped).
constexpr int kMaxLanes = 64;

std::atomic<int> g_load[kMaxLanes];  // calls in progress per lane
std::atomic<unsigned> g_rr{0};
std::atomic<uint64_t> g_spread{0};   // lanes host calls spread over; 0: the caller's device

int lane_count() {
  const int ndev = (int)host_devices().size();
  const int want = knobs().hostq_lanes > 0 ? knobs().hostq_lanes : ndev;
  return want < 1 ? 1 : (want > kMaxLanes ? kMaxLanes : want);
}

int lane_device(int lane) {
  const std::vector<int>& d = host_devices();
  return d[(size_t)lane % d.size()];
}

// The lane in `mask` with the fewest calls in progress, ties broken
// round-robin.
int least_loaded(uint64_t mask) {
  const int n = lane_count();
  const unsigned start = g_rr.fetch_add(1, std::memory_order_relaxed);
  int best = -1, best_load = 0;
  for (int i = 0; i < n; ++i) {
    const int l = (int)((start + (unsigned)i) % (unsigned)n);
    if (!((mask >> l) & 1u)) continue;
    const int x = g_load[l].load(std::memory_order_relaxed);
    if (best < 0 || x < best_load) {
      best = l;
      best_load = x;
      if (x == 0) break;
    }
  }
  return best;
}

// The lane for this call: see above.  LEOEC_E_NO_DEVICE when the caller's
// current device is not one of the gfx950 devices.
int pick_lane(int* lane) {
  if (knobs().hostq_lanes > 0) {
    const int n = lane_count();
    *lane = least_loaded(n >= 64 ? ~0ull : ((1ull << n) - 1));
    return LEOEC_OK;
  }
  const uint64_t spread = g_spread.load(std::memory_order_acquire);
  if (spread) {
    *lane = least_loaded(spread);
    return *lane >= 0 ? LEOEC_OK : LEOEC_E_NO_DEVICE;
  }
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return LEOEC_E_HIP;
  const std::vector<int>& d = host_devices();
  for (size_t i = 0; i < d.size(); ++i)
    if (d[i] == dev) {
      *lane = (int)i;
      return LEOEC_OK;
    }
  return LEOEC_E_NO_DEVICE;
}

// Build lane `lane`'s queue: every slot's buffers up front, each touched once
// by a copy each way (the first transfer through a new pinned buffer costs
// milliseconds, which a caller should not pay inside the queue's lock).
// nullptr when pinned or device memory is short (the lane then has no
// batching: its calls take the per-thread path; the partial queue is
// leaked, as queues are).
Queue* build_queue(int lane) {
  const int dev = lane_device(lane);
  DeviceScope on(dev);
  if (!on.ok()) return nullptr;
  Queue* q = new Queue;
  q->device = dev;
  if (hipStreamCreateWithFlags(&q->up, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&q->down, hipStreamNonBlocking) != hipSuccess)
    return nullptr;
  for (Slot& sl : q->slots) {
    sl.lane = lane;
    sl.up = q->up;
    sl.down = q->down;
    // each arena's first copy on the stream it will use (and the slot's own)
    if (slot_alloc(&sl) != LEOEC_OK ||
        hipMemcpyAsync(sl.d_in, sl.h_in, kSlotBytes, hipMemcpyHostToDevice, q->up) != hipSuccess ||
        hipMemcpyAsync(sl.h_out, sl.d_out, kSlotBytes, hipMemcpyDeviceToHost, q->down) !=
            hipSuccess ||
        hipStreamSynchronize(q->up) != hipSuccess || hipStreamSynchronize(q->down) != hipSuccess ||
        hipMemcpyAsync(sl.d_out, sl.h_out, 4096, hipMemcpyHostToDevice, sl.stream) != hipSuccess ||
        hipStreamSynchronize(sl.stream) != hipSuccess)
      return nullptr;
  }
  std::thread(worker_main, q).detach();
  std::thread(completer_main, q).detach();
  return q;
}

// One queue per lane, built once (~60 ms: 5 x 32 MiB of pinned arenas and
// their device twins) under the lane's own once_flag, so lanes of different
// devices are built concurrently (gf_init / leoec_host_spread warm several
// devices at once) and a caller waits only for the lane it needs.
struct LaneQueue {
  std::once_flag once;
  std::atomic<Queue*> q{nullptr};
};
LaneQueue g_lane_queue[kMaxLanes];
std::atomic<int> g_queues_built{0};

Queue* queue_for(int lane) {
  if (lane < 0 || lane >= kMaxLanes) return nullptr;
  LaneQueue& L = g_lane_queue[lane];
  std::call_once(L.once, [&L, lane] {
    if (Queue* q = build_queue(lane)) {
      L.q.store(q, std::memory_order_release);
      g_queues_built.fetch_add(1, std::memory_order_relaxed);
    }
  });
  return L.q.load(std::memory_order_acquire);
}

}  // namespace

HostqTicket::~HostqTicket() {
  if (queue) {
    Queue* q = static_cast<Queue*>(queue);
    std::lock_guard<std::mutex> lock(q->mu);
    --q->direct;
  }
  if (lane >= 0) g_load[lane].fetch_sub(1, std::memory_order_relaxed);
}

int hostq_lanes() { return device_init() == LEOEC_OK ? lane_count() : 0; }

void hostq_warm(int dev) {
  if (device_init() != LEOEC_OK || !knobs().host_batch) return;
  const int n = lane_count();
  for (int l = 0; l < n; ++l)
    if (lane_device(l) == dev) (void)queue_for(l);
}

bool hostq_queue_ready(int dev) {
  if (device_init() != LEOEC_OK) return false;
  const int n = lane_count();
  bool any = false;
  for (int l = 0; l < n; ++l)
    if (lane_device(l) == dev) {
      if (!g_lane_queue[l].q.load(std::memory_order_acquire)) return false;
      any = true;
    }
  return any;
}

int hostq_queues_built() { return g_queues_built.load(std::memory_order_relaxed); }

int hostq_spread(const int* devices, int n) {
  int rc = device_init();
  if (rc) return rc;
  if (n < 0 || (n > 0 && !devices)) return LEOEC_E_ARG;
  const std::vector<int>& d = host_devices();
  uint64_t mask = 0;
  for (int i = 0; i < n; ++i) {
    size_t j = 0;
    while (j < d.size() && d[j] != devices[i]) ++j;
    if (j == d.size()) return LEOEC_E_NO_DEVICE;  // not a gfx950 device of this process
    mask |= 1ull << j;
  }
  g_spread.store(mask, std::memory_order_release);
  int lanes = 0;
  for (uint64_t x = mask; x; x &= x - 1) ++lanes;
  return lanes;
}

int hostq_run(const HostJob& job, HostqTicket* ticket, void (*overlap)(void*), void* arg) {
  int rc = device_init();
  if (rc) return rc;
  int lane = -1;
  if ((rc = pick_lane(&lane))) return rc;
  g_load[lane].fetch_add(1, std::memory_order_relaxed);
  ticket->lane = lane;  // charged until the call returns (~HostqTicket)
  ticket->device = lane_device(lane);
  if (!knobs().host_batch) return kNotBatched;
  const uint64_t a_in = align_up(job.in_bytes), a_out = align_up(job.out_bytes);
  if (a_in == 0 || a_out == 0 || a_in > kBatchMaxJobBytes || a_out > kBatchMaxJobBytes)
    return kNotBatched;
  Queue* q = queue_for(lane);
  if (!q) return kNotBatched;

  const Clock::time_point t0 = Clock::now();
  std::unique_lock<std::mutex> lk(q->mu);
  if (q->direct < job.direct_cap && (!q->open || q->open->reserved == 0) &&
      q->closed.empty() && q->inflight.empty()) {
    ++q->direct;  // idle queue, few callers: the per-thread path
    ticket->queue = q;
    return kNotBatched;
  }
  // a batch's capacity (Knobs::hostq_slot_kib, at most the arenas); an empty
  // slot takes any batchable job
  const uint64_t cap = std::min<uint64_t>(kSlotBytes, (uint64_t)knobs().hostq_slot_kib << 10);
  Slot* s;
  for (;;) {
    s = q->open;
    if (s && s->jobs.size() < kMaxJobs &&
        (s->jobs.empty() || (s->used_in + a_in <= cap && s->used_out + a_out <= cap)))
      break;
    if (s) {  // full: hand it to the worker, open another
      s->state = St::kClosed;
      q->closed.push_back(s);
      q->nclosed.fetch_add(1, std::memory_order_release);
      q->open = nullptr;
      q->cv_worker.notify_one();
    }
    Slot* f = nullptr;
    for (Slot& x : q->slots)
      if (x.state == St::kFree) {
        f = &x;
        break;
      }
    if (!f) {
      ++q->free_waiters;
      q->cv_free.wait(lk);
      --q->free_waiters;
      continue;
    }
    f->state = St::kOpen;
    f->used_in = f->used_out = 0;
    f->jobs.clear();
    f->in_off.clear();
    f->out_off.clear();
    f->job_rc.clear();
    f->reserved = f->filled = f->readers = 0;
    f->status = LEOEC_OK;
    f->opened = std::chrono::steady_clock::now();
    q->open = f;
  }
  stat_add(9, us_since(t0));
  const uint64_t oi = s->used_in, oo = s->used_out;
  const size_t idx = s->jobs.size();
  s->used_in += a_in;
  s->used_out += a_out;
  s->jobs.push_back(&job);
  s->job_rc.push_back(LEOEC_OK);
  s->in_off.push_back(oi);
  s->out_off.push_back(oo);
  ++s->reserved;
  ++s->readers;
  // the worker waits for an open slot's FIRST reservation (or a closed
  // slot, or room on the GPU, notified where they happen)
  const bool wake = knobs().hostq_wake == 1;
  bool notify = !wake || s->reserved == 1;
  if (knobs().hostq_eager && (s->used_in + a_in > cap || s->used_out + a_out > cap ||
                              s->jobs.size() >= kMaxJobs)) {
    // no room for another job of this size: the batch is complete, so it
    // goes to the worker now, and its H2D queues behind the previous
    // batch's instead of starting after it ends (tools/copy_gaps.py: at
    // every gap of the H2D stream the previous batch alone was on the GPU)
    s->state = St::kClosed;
    q->closed.push_back(s);
    q->nclosed.fetch_add(1, std::memory_order_release);
    q->open = nullptr;
    notify = true;
  }
  if (notify) q->cv_worker.notify_one();
  lk.unlock();

  const bool gather = job.in.size() > 1;
  for (const HostSeg& g : job.in) pack_pinned(s->h_in + oi + g.off, g.src, g.n, gather);
  // bytes of the region no segment covers are read by the kernels only
  // inside an aligned 16-byte chunk that also holds real bytes, and cleared
  // there (kernels_impl.hpp guarded tiles): nothing to zero

  lk.lock();
  if (++s->filled == s->reserved) q->cv_worker.notify_one();
  lk.unlock();
  if (overlap) overlap(arg);
  lk.lock();
  const Clock::time_point tw = Clock::now();
  if (wake) {
    s->cv_done.wait(lk, [s] { return s->state == St::kDone; });
  } else {
    ++q->done_waiters;
    q->cv_done.wait(lk, [s] { return s->state == St::kDone; });
    --q->done_waiters;
  }
  stat_add(8, us_since(tw));
  const int status = s->status != LEOEC_OK ? s->status : s->job_rc[idx];
  lk.unlock();
  if (status == LEOEC_OK)
    for (const OutSeg& g : job.out) std::memcpy(g.dst, s->h_out + oo + g.off, g.n);
  lk.lock();
  if (--s->readers == 0) {
    stat_add(7, us_since(s->done));
    s->state = St::kFree;
    if (q->free_waiters > 0) q->cv_free.notify_all();
  }
  return status;
}

}  // namespace leoec

#ifdef LEOEC_MEASURE
// Measurement build: the queue's timeline counters since the last call
// (batches, jobs, launches, then summed microseconds: worker waiting for
// fills, issuing copies + launches, completer waiting on the GPU, slot open
// until closed, DONE until FREE, callers waiting for DONE, callers waiting
// to reserve).  Resets them.
extern "C" __attribute__((visibility("default"))) void leoec_measure_hostq_stats(double* out14) {
  std::lock_guard<std::mutex> l(leoec::g_stats.mu);
  for (int i = 0; i < 14; ++i) {
    out14[i] = leoec::g_stats.v[i];
    leoec::g_stats.v[i] = 0;
  }
}

// Measurement build: jobs launched per dispatcher lane since the last call
// (batched jobs only); resets them.
extern "C" __attribute__((visibility("default"))) void leoec_measure_hostq_lane_jobs(double* out64) {
  std::lock_guard<std::mutex> l(leoec::g_stats.mu);
  for (int i = 0; i < 64; ++i) {
    out64[i] = leoec::g_lane_jobs[i];
    leoec::g_lane_jobs[i] = 0;
  }
}
#endif
