// engine.hpp — host side of the engine: code cache, survivor selection,
// decoding maps, device context and the operations behind the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
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

// Enqueue "out blocks = map(survivor blocks)" for a batch.  in: k shards in
// survivor order; out: nwant shards.
int apply(const Code& c, const int* surv, const std::vector<Shard>& in, const int* want,
          const std::vector<Shard>& out, uint64_t block_size, uint64_t nobj, hipStream_t s);

int device_init();  // opens the HIP device once; LEOEC_E_NO_DEVICE if unusable

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

}  // namespace leoec
