// hostq.cpp — see hostq.hpp.
//
// Per device: kSlots batch slots, each a pinned input arena + pinned output
// arena + their device twins, a stream and an event.  A slot moves
//   FREE -> OPEN (callers reserve space and copy their inputs in)
//        -> CLOSED (no more reservations; the worker waits for the copies)
//        -> INFLIGHT (H2D, launches, D2H enqueued on the slot's stream)
//        -> DONE (callers copy their outputs out) -> FREE (last reader).
// The worker closes the open slot whenever fewer than Knobs::hostq_depth
// batches are on the GPU, so calls arriving while the GPU is busy pile into
// one batch, and a lone call is launched at once.  The completer thread waits for batches
// in launch order and wakes their callers.
#include "hostq.hpp"

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

#include "../../include/leoec.h"
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
#else
inline void stat_add(int, double) {}
#endif

enum class St { kFree, kOpen, kClosed, kInflight, kDone };

struct Slot {
  St state = St::kFree;
  bool ready = false;  // buffers, stream and event exist
  uint8_t* h_in = nullptr;
  uint8_t* h_out = nullptr;
  uint8_t* d_in = nullptr;
  uint8_t* d_out = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev = nullptr;
  hipEvent_t ev_h2d = nullptr;  // after the input copy: the H2D engine is free for the next batch
  uint64_t used_in = 0, used_out = 0;
  std::vector<const HostJob*> jobs;
  std::vector<uint64_t> in_off, out_off;
  int reserved = 0, filled = 0, readers = 0;
  int status = LEOEC_OK;
  Clock::time_point opened, done;
};

struct Queue {
  int device = -1;
  std::mutex mu;
  std::condition_variable cv_worker;    // work for the worker (jobs, fills, GPU room)
  std::condition_variable cv_complete;  // work for the completer
  std::condition_variable cv_free;      // a slot became FREE
  std::condition_variable cv_done;      // a slot became DONE
  Slot slots[kSlots];
  Slot* open = nullptr;
  std::deque<Slot*> closed;    // closed by a caller because it was full
  std::deque<Slot*> inflight;  // launch order
  Slot* last = nullptr;        // most recently launched
  int direct = 0;              // calls on their per-thread path (HostqTicket)
};

// Wait for `ev` without holding the queue lock: hipEventSynchronize, or
// (Knobs::hostq_sync = 1, measurement) a hipEventQuery poll with yields.
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

int slot_alloc(Slot* s) {
  if (hipHostMalloc((void**)&s->h_in, kSlotBytes, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&s->h_out, kSlotBytes, hipHostMallocDefault) != hipSuccess ||
      hipMalloc((void**)&s->d_in, kSlotBytes) != hipSuccess ||
      hipMalloc((void**)&s->d_out, kSlotBytes) != hipSuccess ||
      hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->ev_h2d, hipEventDisableTiming) != hipSuccess) {
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
  return a.code == b.code && a.bs == b.bs && a.in_blk == b.in_blk && a.out_blk == b.out_blk &&
         a.out_valid == b.out_valid && a.in_bytes == b.in_bytes && a.out_bytes == b.out_bytes &&
         a.surv == b.surv && a.want == b.want && a.in_valid == b.in_valid;
}

// Enqueue one batch: ONE H2D of the input arena, one launch per run of
// consecutive identical maps (their regions are uniformly strided: they were
// reserved back to back with the same sizes), ONE D2H of the output arena.
// The event is recorded whatever happened, so the completer always waits
// for the work that was enqueued before the slot can be reused.
int launch_slot(Slot* s) {
  Clock::time_point t = Clock::now();
  int rc = hipMemcpyAsync(s->d_in, s->h_in, s->used_in, hipMemcpyHostToDevice, s->stream) ==
                   hipSuccess
               ? LEOEC_OK
               : LEOEC_E_HIP;
  if (rc == LEOEC_OK && hipEventRecord(s->ev_h2d, s->stream) != hipSuccess) rc = LEOEC_E_HIP;
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
    const int k = (int)J.surv.size(), r = (int)J.want.size();
    std::vector<Shard> in(k), out(r);
    for (int b = 0; b < k; ++b)
      in[b] = Shard{s->d_in + s->in_off[i] + (uint64_t)b * J.in_blk, sin, J.in_valid[b]};
    for (int o = 0; o < r; ++o)
      out[o] = Shard{s->d_out + s->out_off[i] + (uint64_t)o * J.out_blk, sout, J.out_valid};
    rc = apply(*J.code, J.surv.data(), in, J.want.data(), out, J.bs, (uint64_t)(j - i), s->stream);
    stat_add(2, 1);
    i = j;
  }
  stat_add(12, us_since(t));
  t = Clock::now();
  if (rc == LEOEC_OK &&
      hipMemcpyAsync(s->h_out, s->d_out, s->used_out, hipMemcpyDeviceToHost, s->stream) !=
          hipSuccess)
    rc = LEOEC_E_HIP;
  stat_add(13, us_since(t));
  if (hipEventRecord(s->ev, s->stream) != hipSuccess) {
    (void)hipStreamSynchronize(s->stream);  // no event to wait on: drain here
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
      (void)wait_event(prev->ev_h2d);
      lk.lock();
      q->last = nullptr;
      continue;
    }
    Slot* s;
    if (!q->closed.empty()) {
      s = q->closed.front();
      q->closed.pop_front();
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
    const int rc = wait_event(s->ev) == hipSuccess ? LEOEC_OK : LEOEC_E_HIP;
    stat_add(5, us_since(tw));
    lk.lock();
    s->done = Clock::now();
    q->inflight.pop_front();
    if (q->last == s) q->last = nullptr;
    if (s->status == LEOEC_OK) s->status = rc;
    s->state = St::kDone;
    q->cv_done.notify_all();
    q->cv_worker.notify_one();
  }
}

// One queue per device, created on first use; its two threads live for the
// process (they hold no GPU work when idle, and a process exits with them
// parked on their condition variables).
constexpr int kMaxDevices = 64;

Queue* queue_for(int dev) {
  static std::mutex mu;
  static Queue* queues[kMaxDevices] = {};
  static bool failed[kMaxDevices] = {};
  if (dev < 0 || dev >= kMaxDevices) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!queues[dev] && !failed[dev]) {
    // every slot's buffers up front, each touched once by a copy each way:
    // the first transfer through a new pinned buffer costs milliseconds,
    // which a caller should not pay inside the queue's lock
    Queue* q = new Queue;
    q->device = dev;
    for (Slot& sl : q->slots) {
      if (slot_alloc(&sl) != LEOEC_OK ||
          hipMemcpyAsync(sl.d_in, sl.h_in, kSlotBytes, hipMemcpyHostToDevice, sl.stream) !=
              hipSuccess ||
          hipMemcpyAsync(sl.h_out, sl.d_out, kSlotBytes, hipMemcpyDeviceToHost, sl.stream) !=
              hipSuccess ||
          hipStreamSynchronize(sl.stream) != hipSuccess) {
        failed[dev] = true;  // no batching on this device (pinned memory short): per-thread path
        return nullptr;      // (the partial queue is leaked, as queues are)
      }
    }
    std::thread(worker_main, q).detach();
    std::thread(completer_main, q).detach();
    queues[dev] = q;
  }
  return queues[dev];
}

}  // namespace

HostqTicket::~HostqTicket() {
  if (!queue) return;
  Queue* q = static_cast<Queue*>(queue);
  std::lock_guard<std::mutex> lock(q->mu);
  --q->direct;
}

int hostq_run(const HostJob& job, HostqTicket* ticket, void (*overlap)(void*), void* arg) {
  if (!knobs().host_batch) return kNotBatched;
  const uint64_t a_in = align_up(job.in_bytes), a_out = align_up(job.out_bytes);
  if (a_in == 0 || a_out == 0 || a_in > kBatchMaxJobBytes || a_out > kBatchMaxJobBytes)
    return kNotBatched;
  int rc = device_init();
  if (rc) return rc;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return LEOEC_E_HIP;
  Queue* q = queue_for(dev);
  if (!q) return kNotBatched;

  const Clock::time_point t0 = Clock::now();
  std::unique_lock<std::mutex> lk(q->mu);
  if (ticket && q->direct < job.direct_cap && (!q->open || q->open->reserved == 0) &&
      q->closed.empty() && q->inflight.empty()) {
    ++q->direct;  // idle queue, few callers: the per-thread path
    ticket->queue = q;
    return kNotBatched;
  }
  Slot* s;
  for (;;) {
    s = q->open;
    if (s && s->used_in + a_in <= kSlotBytes && s->used_out + a_out <= kSlotBytes &&
        s->jobs.size() < kMaxJobs)
      break;
    if (s) {  // full: hand it to the worker, open another
      s->state = St::kClosed;
      q->closed.push_back(s);
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
      q->cv_free.wait(lk);
      continue;
    }
    f->state = St::kOpen;
    f->used_in = f->used_out = 0;
    f->jobs.clear();
    f->in_off.clear();
    f->out_off.clear();
    f->reserved = f->filled = f->readers = 0;
    f->status = LEOEC_OK;
    f->opened = std::chrono::steady_clock::now();
    q->open = f;
  }
  stat_add(9, us_since(t0));
  const uint64_t oi = s->used_in, oo = s->used_out;
  s->used_in += a_in;
  s->used_out += a_out;
  s->jobs.push_back(&job);
  s->in_off.push_back(oi);
  s->out_off.push_back(oo);
  ++s->reserved;
  ++s->readers;
  q->cv_worker.notify_one();
  lk.unlock();

  for (const HostSeg& g : job.in) std::memcpy(s->h_in + oi + g.off, g.src, g.n);
  // bytes of the region no segment covers are read by the kernels only
  // inside an aligned 16-byte chunk that also holds real bytes, and cleared
  // there (kernels_impl.hpp guarded tiles): nothing to zero

  lk.lock();
  if (++s->filled == s->reserved) q->cv_worker.notify_one();
  lk.unlock();
  if (overlap) overlap(arg);
  lk.lock();
  const Clock::time_point tw = Clock::now();
  q->cv_done.wait(lk, [s] { return s->state == St::kDone; });
  stat_add(8, us_since(tw));
  const int status = s->status;
  lk.unlock();
  if (status == LEOEC_OK)
    for (const OutSeg& g : job.out) std::memcpy(g.dst, s->h_out + oo + g.off, g.n);
  lk.lock();
  if (--s->readers == 0) {
    stat_add(7, us_since(s->done));
    s->state = St::kFree;
    q->cv_free.notify_all();
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
#endif
