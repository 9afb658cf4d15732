// capi.cpp — extern "C" entry points of libleoec.so (include/leoec.h).
// No C++ exception crosses this boundary: anything thrown below becomes a
// status code (the reference lets `new std::bad_alloc()` escape its catch
// blocks and take the VM down, c_src/rscoding.cpp:69).
#include <new>

#include "../../include/leoec.h"
#include "engine.hpp"
#include "hostq.hpp"

#define LEOEC_VERSION "0.1.0"

namespace {

template <typename F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return LEOEC_E_NOMEM;
  } catch (...) {
    return LEOEC_E_ARG;
  }
}

}  // namespace

extern "C" {

const char* leoec_strerror(int status) {
  switch (status) {
    case LEOEC_OK: return "ok";
    case LEOEC_E_INVALID_CODING: return "Invalid Coding";
    case LEOEC_E_PARAMS: return "Invalid Coding Parameters";
    case LEOEC_E_PARAMS_W_RS: return "Invalid Coding Parameters (w = 8/16/32)";
    case LEOEC_E_PARAMS_LARGER_W: return "Invalid Coding Parameters (larger w)";
    case LEOEC_E_PARAMS_M2: return "Invalid Coding Parameters (m = 2)";
    case LEOEC_E_PARAMS_K_LE_W: return "Invalid Coding Parameters (k <= w)";
    case LEOEC_E_PARAMS_W_PRIME: return "Invalid Coding Parameters (w is prime)";
    case LEOEC_E_PARAMS_W8: return "Invalid Coding Parameters (w = 8)";
    case LEOEC_E_NOT_ENOUGH_BLOCKS: return "Not Enough Blocks";
    case LEOEC_E_NOT_UNIQUE: return "Blocks should be unique";
    case LEOEC_E_NON_INVERTIBLE: return "Non Invertible";
    case LEOEC_E_BAD_ID: return "Invalid Block ID";
    case LEOEC_E_BAD_SIZE: return "Invalid Block Size";
    case LEOEC_E_UNSUPPORTED: return "Unsupported Coding Parameters";
    case LEOEC_E_NOMEM: return "Out of Memory";
    case LEOEC_E_NO_DEVICE: return "No gfx950 HIP device";
    case LEOEC_E_HIP: return "HIP runtime error";
    case LEOEC_E_ARG: return "Invalid Argument";
    default: return "Unknown Error";
  }
}

// gf_init/0 (nif.cpp:122-128): the field tables, then the device runtime
// warmed on the caller's current device (engine.cpp warm_device), so the
// VM's first encode does not pay the runtime's lazy set-up.
int leoec_gf_init(void) {
  return guarded([] {
    for (int w : {8, 16, 32}) (void)leoec::field(w);
    const int rc = leoec::device_init();
    if (rc == LEOEC_OK) (void)leoec::warm_current_device();
    return rc;
  });
}

int leoec_check_params(int coding, int k, int m, int w) {
  return leoec::check_params(coding, k, m, w);
}

int leoec_layout(int coding, int k, int m, int w, uint64_t size, uint64_t* block_size,
                 int* filled) {
  return guarded([&] { return leoec::op_layout(coding, k, m, w, size, block_size, filled); });
}

int leoec_encode(int coding, int k, int m, int w, const uint8_t* obj, uint64_t size, uint8_t* out,
                 uint64_t out_size) {
  return guarded([&] { return leoec::op_encode(coding, k, m, w, obj, size, out, out_size); });
}

int leoec_decode(int coding, int k, int m, int w, const uint8_t* const* blocks, const int* ids,
                 int nblocks, uint64_t block_size, uint64_t size, uint8_t* out) {
  return guarded([&] {
    return leoec::op_decode(coding, k, m, w, blocks, ids, nblocks, block_size, size, out);
  });
}

int leoec_repair(int coding, int k, int m, int w, const uint8_t* const* blocks, const int* ids,
                 int nblocks, uint64_t block_size, const int* repair_ids, int nrepair,
                 uint8_t* out) {
  return guarded([&] {
    return leoec::op_repair(coding, k, m, w, blocks, ids, nblocks, block_size, repair_ids,
                            nrepair, out);
  });
}

int leoec_encode_dev(int coding, int k, int m, int w, const uint8_t* objs, uint64_t obj_stride,
                     uint64_t size, uint64_t nobj, uint8_t* parity, uint64_t parity_stride,
                     void* stream) {
  return guarded([&] {
    return leoec::op_encode_dev(coding, k, m, w, objs, obj_stride, size, nobj, parity,
                                parity_stride, (hipStream_t)stream);
  });
}

int leoec_decode_dev(int coding, int k, int m, int w, uint8_t* objs, uint64_t obj_stride,
                     uint64_t size, uint64_t nobj, const uint8_t* parity, uint64_t parity_stride,
                     const int* erased, int nerased, void* stream) {
  return guarded([&] {
    return leoec::op_decode_dev(coding, k, m, w, objs, obj_stride, size, nobj, parity,
                                parity_stride, erased, nerased, (hipStream_t)stream);
  });
}

int leoec_repair_dev(int coding, int k, int m, int w, const uint8_t* const* blocks,
                     uint64_t block_stride, uint64_t block_size, uint64_t nobj,
                     const int* repair_ids, int nrepair, uint8_t* const* out,
                     uint64_t out_stride, void* stream) {
  return guarded([&] {
    return leoec::op_repair_dev(coding, k, m, w, blocks, block_stride, block_size, nobj,
                                repair_ids, nrepair, out, out_stride, (hipStream_t)stream);
  });
}

int leoec_coding_matrix(int coding, int k, int m, int w, uint32_t* out, int cap, int* n_out) {
  return guarded([&] {
    const leoec::Code* c;
    int rc = leoec::get_code(coding, k, m, w, &c);
    if (rc) return rc;
    if (!c->bitmatrix) {
      const int n = (int)c->C.a.size();
      if (n_out) *n_out = n;
      if (!out || cap < n) return (int)LEOEC_E_ARG;
      for (int i = 0; i < n; ++i) out[i] = c->C.a[i];
      return (int)LEOEC_OK;
    }
    const int n = c->B.rows * c->B.cols;
    if (n_out) *n_out = n;
    if (!out || cap < n) return (int)LEOEC_E_ARG;
    for (int r = 0; r < c->B.rows; ++r)
      for (int col = 0; col < c->B.cols; ++col) out[r * c->B.cols + col] = c->B.get(r, col);
    return (int)LEOEC_OK;
  });
}

int leoec_device(void) {
  return guarded([] {
    int rc = leoec::device_init();
    if (rc) return rc;
    int dev = 0;
    return hipGetDevice(&dev) == hipSuccess ? dev : (int)LEOEC_E_HIP;
  });
}

int leoec_host_lanes(int* devices, int cap) {
  return guarded([&] {
    int rc = leoec::device_init();
    if (rc) return rc;
    const int n = leoec::hostq_lanes();
    const std::vector<int>& d = leoec::host_devices();
    for (int i = 0; devices && i < n && i < cap; ++i) devices[i] = d[(size_t)i % d.size()];
    return n;
  });
}

// The set's devices are warmed before this returns (engine.cpp
// warm_devices): a device's first call then neither creates its hardware
// queues nor its lane's batching queue behind the callers.
int leoec_host_spread(const int* devices, int n) {
  return guarded([&] {
    const int rc = leoec::hostq_spread(devices, n);
    if (rc > 0) leoec::warm_devices(devices, n);
    return rc;
  });
}

const char* leoec_version(void) { return LEOEC_VERSION " (gfx950)"; }

}  // extern "C"
