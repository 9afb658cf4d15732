// engine.hpp — host side of the engine: code cache, survivor selection,
// decoding maps, device context and the operations behind the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <vector>

#include "codes.hpp"
#include "kernels.hpp"

namespace leoec {

// The coding class resolved for (coding, k, m, w): either a GF(2^w) coding
// matrix (vandrs, isars) or a GF(2) coding bitmatrix (cauchyrs, liberation).
struct Code {
  int coding = 0, k = 0, m = 0, w = 0;
  bool bitmatrix = false;
  GfMatrix C;   // m x k
  BitMatrix B;  // (m*w) x (k*w)
};

int check_params(int coding, int k, int m, int w);
int get_code(int coding, int k, int m, int w, const Code** out);  // cached

// Rows expressing the `want` block ids in terms of the k survivor ids `surv`
// (the reference's decoding matrices; see engine.cpp).
int gf_rows(const Code& c, const int* surv, const int* want, int nwant, std::vector<uint32_t>* rows);
int bit_rows(const Code& c, const int* surv, const int* want, int nwant, std::vector<uint8_t>* rows);

// The map "out blocks = f(survivor blocks)" of one (code, survivors,
// wanted ids), built on the host once: GF(2^w) coefficient rows (vandrs,
// isars, cauchyrs through the packet-bitsliced kernel), GF(2) bit rows (the
// generic bitmatrix kernel) or liberation's syndrome-decode masks.  All the
// host arithmetic of a call (the k x k / kw x kw inversions) happens here, so
// a plan that fails fails on the calling thread, before any device work.
struct Plan {
  enum Kind { kGf, kGfBit, kLibDec, kBit };
  Kind kind = kGf;
  const Code* code = nullptr;
  std::vector<int> surv, want;
  std::vector<uint32_t> coef;   // kGf, kGfBit: nwant x k
  std::vector<uint8_t> bits;    // kBit: (nwant w) x (k w)
  std::vector<int> lib_pos;     // kLibDec: id -> index of its shard in `in` (k + 2), -1 absent
  std::vector<uint32_t> mbits;  // kLibDec: nwant x 2w
};

// Cached by (code, survivors, wanted ids): repeated erasure patterns reuse
// their inverse.  The shared_ptr keeps a plan alive while a batch uses it.
int make_plan(const Code& c, const int* surv, const int* want, int nwant,
              std::shared_ptr<const Plan>* out);
// Host bytes a plan holds (its tables): the plan cache's size bound.
size_t plan_bytes(const Plan& p);
// Enqueue a plan over a batch.  in: k shards in survivor order; out: nwant.
int run_plan(const Plan& p, const std::vector<Shard>& in, const std::vector<Shard>& out,
             uint64_t block_size, uint64_t nobj, hipStream_t s);
// make_plan + run_plan.
int apply(const Code& c, const int* surv, const std::vector<Shard>& in, const int* want,
          const std::vector<Shard>& out, uint64_t block_size, uint64_t nobj, hipStream_t s);

// Opens the HIP runtime once and lists its gfx950 devices; LEOEC_E_NO_DEVICE
// if there is none.
int device_init();
// The gfx950 device ordinals the host-memory entry points spread their calls
// over (valid after device_init() returned LEOEC_OK).
const std::vector<int>& host_devices();
constexpr int kMaxDevices = 64;

// Makes `dev` the calling thread's current HIP device for a scope and puts
// the previous one back (host-memory calls run on the device the dispatcher
// picked without changing the caller's own device).
class DeviceScope {
 public:
  explicit DeviceScope(int dev);
  ~DeviceScope();
  bool ok() const { return ok_; }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;

 private:
  int prev_ = -1;
  bool ok_ = true;
};

// Operations behind the C ABI (argument checking included).
int op_layout(int coding, int k, int m, int w, uint64_t size, uint64_t* bs, int* filled);
int op_encode(int coding, int k, int m, int w, const uint8_t* obj, uint64_t size, uint8_t* out,
              uint64_t out_size);
int op_decode(int coding, int k, int m, int w, const uint8_t* const* blocks, const int* ids, int n,
              uint64_t bs, uint64_t size, uint8_t* out);
int op_repair(int coding, int k, int m, int w, const uint8_t* const* blocks, const int* ids, int n,
              uint64_t bs, const int* rep, int nrep, uint8_t* out);
int op_encode_dev(int coding, int k, int m, int w, const uint8_t* objs, uint64_t obj_stride,
                  uint64_t size, uint64_t nobj, uint8_t* parity, uint64_t parity_stride,
                  hipStream_t s);
int op_decode_dev(int coding, int k, int m, int w, uint8_t* objs, uint64_t obj_stride,
                  uint64_t size, uint64_t nobj, const uint8_t* parity, uint64_t parity_stride,
                  const int* erased, int nerased, hipStream_t s);
int op_repair_dev(int coding, int k, int m, int w, const uint8_t* const* blocks,
                  uint64_t block_stride, uint64_t bs, uint64_t nobj, const int* rep, int nrep,
                  uint8_t* const* out, uint64_t out_stride, hipStream_t s);

// The runtime warm-up of one device (once per device; best effort, always
// LEOEC_OK): hardware queues, the pageable-copy staging, every kernel code
// object, the device's batching queue and its pools of per-thread streams
// and mapped buffers.  gf_init warms the caller's current device;
// leoec_host_spread warms every device of its set (warm_devices, one thread
// per device).
int warm_device(int dev);
int warm_current_device();
void warm_devices(const int* devs, int n);

// What the warm-up left on a device (tests): pooled streams and mapped
// buffers not yet taken by a thread, whether every lane of the device has
// its batching queue, and the process's count of built queues.
struct WarmState {
  int pool_streams = 0;
  int pool_mapped = 0;
  bool queue = false;
  int queues_built = 0;
};
WarmState warm_state(int dev);

// The per-thread staging of exited threads (engine.cpp Staging::hand_off,
// reclaim_drain): stagings handed off at thread exit, stagings freed by a
// live thread, and handed-off stagings found with work in flight (the
// invariant says none); and warm_devices' threads started / finished.
struct ReclaimState {
  long handed_off = 0;
  long drained = 0;
  long busy = 0;
  long warm_threads_started = 0;
  long warm_threads_done = 0;
};
ReclaimState reclaim_state();

}  // namespace leoec
