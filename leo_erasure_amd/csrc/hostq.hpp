// hostq.hpp — cross-call batching of the host-memory entry points.
//
// The reference is called once per object, from many scheduler threads at
// once (basho_bench {concurrent, 4}: test/basho_bench_leo_erasure_rs_10_4_8_
// 1M_w_t4.config:24), and every call starts and ends in host memory
// (c_src/rscoding.cpp:41,73-81).  One PCIe round trip per object costs
// ~15-20 us of copy submit + wait per copy whatever its size, so concurrent
// calls are packed: each device has a queue whose worker thread takes every
// call that arrived while the previous batch was on the GPU, and moves the
// batch with ONE H2D, one launch per run of identical maps (nobj > 1), and
// ONE D2H.  Callers pack their own inputs into the batch's pinned buffer and
// unpack their outputs (host memcpys run in parallel on the callers'
// threads); the worker only issues copies and launches.  A lone caller pays
// no window: a batch closes as soon as the GPU has room for it.
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

#include "engine.hpp"

namespace leoec {

struct HostSeg {  // caller buffer -> job input region
  const uint8_t* src;
  uint64_t off, n;
};
struct OutSeg {  // job output region -> caller buffer
  uint8_t* dst;
  uint64_t off, n;
};

// One call's map: out block o = map(surv -> want[o]) applied to k input
// blocks.  Input block i lives at in_blk * i inside the job's input region
// (in_valid[i] bytes of it are real, the rest read as zero), output block o
// at out_blk * o inside its output region.
struct HostJob {
  std::shared_ptr<const Plan> plan;  // built on the caller's thread (engine.hpp make_plan)
  uint64_t bs = 0;  // kernel block geometry (multiple of 16)
  uint64_t in_blk = 0, out_blk = 0;
  std::vector<uint64_t> in_valid;  // per input block
  uint64_t out_valid = 0;          // per output block
  uint64_t in_bytes = 0, out_bytes = 0;
  std::vector<HostSeg> in;
  std::vector<OutSeg> out;
  int direct_cap = 0;  // calls of this kind allowed on the per-thread path at an idle queue
};

// Largest job input / output region that is batched; larger calls take the
// per-thread path (their copies amortise their own submit cost).
constexpr uint64_t kBatchMaxJobBytes = (uint64_t)8 << 20;

// Held by a call that hostq_run sent to its per-thread path: `device` is the
// device it runs on (the dispatcher's pick; -1: the caller's current
// device), and the call counts against that device's load until it returns.
struct HostqTicket {
  int device = -1;
  int lane = -1;         // dispatcher lane (logical queue) charged with the call
  void* queue = nullptr; // set when the call holds one of the queue's direct places
  HostqTicket() = default;
  HostqTicket(const HostqTicket&) = delete;
  HostqTicket& operator=(const HostqTicket&) = delete;
  ~HostqTicket();
};

// Run `job` and wait for it: on the caller's current device by default, or,
// after hostq_spread(), on the lane (one queue per device; the measurement
// build can map more lanes onto fewer devices) of the spread set with the
// fewest calls in progress, ties taken round-robin, so concurrent callers
// spread over those devices and their PCIe links.  `overlap` (may be null) runs on the
// caller's thread while the batch is on the GPU.  Returns a leoec_status
// (this job's own: another caller's failed launch does not fail it), or
// kNotBatched: nothing was done and the caller runs its per-thread path on
// ticket->device — the job is too large, batching is off, pinned memory is
// short, or the lane's queue is idle and fewer than job.direct_cap calls are
// already running direct.
constexpr int kNotBatched = 1;
int hostq_run(const HostJob& job, HostqTicket* ticket, void (*overlap)(void*) = nullptr,
              void* arg = nullptr);

// Dispatcher lanes (one per gfx950 device in the product build), or 0
// without a device.
int hostq_lanes();

// Warm-up (gf_init, leoec_host_spread): creates the batching queue of every
// lane on device `dev` now (its pinned arenas and threads: ~60 ms), rather
// than inside the first batchable call.
void hostq_warm(int dev);

// Whether every lane of device `dev` has its queue (tests: the warm-up made
// them), and how many queues this process has built.
bool hostq_queue_ready(int dev);
int hostq_queues_built();

// leoec_host_spread: spread host-memory calls over these device ordinals
// (n > 0), or run each on the caller's current device again (n == 0).
// Returns the number of lanes in the set or a negative status.
int hostq_spread(const int* devices, int n);

}  // namespace leoec
