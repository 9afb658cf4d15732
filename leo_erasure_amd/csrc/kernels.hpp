// kernels.hpp — launch interface of the gfx950 kernels (kernels.hip).
//
// Every coding operation of the engine is one of two linear maps applied
// column-by-column to a batch of objects:
//   * GfApply  — out_r = XOR_j C[r][j] * in_j over GF(2^w), w in {8,16,32},
//                byte-wise (w=8) or on little-endian words (w=16/32):
//                jerasure_matrix_encode / _decode_data / _decode_selected and
//                ISA-L ec_encode_data (c_src/rscoding.cpp:71,147,198,
//                c_src/irscoding.cpp:70,134,176);
//   * BitApply — out packet o = XOR of in packets p with B[o][p] = 1, packet
//                = block_size / w bytes: jerasure_schedule_encode and the lazy
//                schedule decoders (c_src/cauchycoding.cpp:72,149,199,
//                c_src/liberationcoding.cpp:72,147,195).
// A "shard" is one block of every object in the batch: block of object o at
// base + o * stride; bytes at offset >= valid are read as zero / not written.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace leoec {

struct Shard {
  const uint8_t* base;
  uint64_t stride;
  uint64_t valid;
};

struct GfApply {
  int w = 8;
  int K = 0, R = 0;
  std::vector<uint32_t> coef;  // R x K, row-major
  std::vector<Shard> in, out;  // K / R shards
  uint64_t block_size = 0;     // bytes per block (multiple of 16)
  uint64_t nobj = 0;
};

struct BitApply {
  int w = 0;
  int KB = 0, RB = 0;           // input / output blocks
  std::vector<uint8_t> bits;    // (RB*w) x (KB*w), row-major 0/1
  std::vector<Shard> in, out;   // KB / RB shards
  uint64_t block_size = 0;      // multiple of 16*w (packet = block_size / w)
  uint64_t nobj = 0;
};

// A GF(2^w) matrix applied to packet-bitsliced blocks: block = w packets of
// block_size / w bytes, packet x holding bit x of every symbol.  This is the
// bitmatrix product of the matrix's bit expansion (cauchyrs, whose coding
// and decoding bitmatrices are expansions of GF(2^w) matrices), computed as
// sum over set coefficient bits t of (block * 2^t), with *2 done on packets.
struct GfBitApply {
  int w = 0;
  int K = 0, R = 0;
  std::vector<uint32_t> coef;  // R x K
  std::vector<Shard> in, out;
  uint64_t block_size = 0;     // multiple of 16*w
  uint64_t nobj = 0;
};

// Liberation decode / repair of erased data blocks through syndromes
// (kernels_impl.hpp lib_dec_apply): data[j] = surviving data block j (base
// nullptr if erased), cod[0..1] = P, Q if survivors; the wanted outputs are
// erased data blocks; mbits[b][s] holds, for wanted block b and syndrome
// packet s (P 0..w-1, Q w..2w-1), bit 31-x set when s feeds packet x.
struct LibDecApply {
  int w = 0, k = 0;
  std::vector<Shard> data, cod, out;  // k, 2, nout (<= 2) shards
  std::vector<uint32_t> mbits;        // nout x 2w
  uint64_t block_size = 0;
  uint64_t nobj = 0;
};

// Enqueue on `stream`; returns a leoec_status.
int launch(const GfApply& plan, hipStream_t stream);
int launch(const BitApply& plan, hipStream_t stream);
int launch(const GfBitApply& plan, hipStream_t stream);
int launch(const LibDecApply& plan, hipStream_t stream);
bool gfbit_supported(int w);
bool lib_dec_supported(int w);  // a lib_dec_apply instance exists and LEOEC_LIB_FORM != 0

}  // namespace leoec
