// xor_pattern.hip — measurement library only (not a code): the access-pattern
// ceiling of the headline encode, for bench.py's roofline.pattern_ceiling
// ("also measure an achievable-copy kernel").
//
// The RS(10,4,8) encode's traffic without its arithmetic: every lane loads
// one 16-byte column of the 10 data blocks of an object (non-temporal raw
// buffer loads, all ten in flight) and stores 4 parity columns, each the XOR
// of the ten.  64-lane workgroups in tile-major order: the fastest of the
// orders tools/order_ceiling.hip measures at 1 MiB (0.80 of 8 TB/s,
// profiles/r03b_v6_order_ceiling.log).  The gf8_apply COPY forms
// (LEOEC_GF8_VARIANT=7/27/39/43) keep gf8_apply's register and LDS shape and
// read 0.72-0.74 on the same box (profiles/r03b_v6_copyforms.log), below the
// shipped kernel itself, so they are not a ceiling.
//
// Geometry as rscoding.cpp:44 (vandrs, w = 8): bs = roundup16(ceil(size /
// (k w))) * w.  Data block j of object o starts at objs + o*stride + j*bs and
// holds min(bs, size - j*bs) bytes (the rest reads as zero through the
// buffer range); parity block r at parity + o*pstride + r*bs.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kK = 10, kR = 4, kLanes = 64;

struct XorArgs {
  const uint8_t* objs;
  uint64_t stride;
  uint8_t* parity;
  uint64_t pstride;
  uint32_t size;
  uint32_t bs;
  uint32_t tiles;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t range(const uint8_t* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), 0, n, 0x00020000);
}

__global__ void __launch_bounds__(kLanes) xor_pattern(const XorArgs a) {
  const uint32_t obj = blockIdx.x / a.tiles;
  const uint32_t off = (blockIdx.x - obj * a.tiles) * (kLanes * 16u) + threadIdx.x * 16u;
  if (off >= a.bs) return;
  const uint8_t* ib = a.objs + (uint64_t)obj * a.stride;
  uint8_t* ob = a.parity + (uint64_t)obj * a.pstride;
  u32x4 d[kK];
#pragma unroll
  for (int j = 0; j < kK; ++j) {
    const uint32_t lo = (uint32_t)j * a.bs;
    const uint32_t valid = a.size > lo ? (a.size - lo < a.bs ? a.size - lo : a.bs) : 0u;
    d[j] = __builtin_amdgcn_raw_buffer_load_b128(range(ib + lo, valid), off, 0, 2);
  }
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    u32x4 acc = d[r];
#pragma unroll
    for (int j = 0; j < kK; ++j)
      if (j != r) acc ^= d[j];
    __builtin_amdgcn_raw_buffer_store_b128(acc, range(ob + (uint64_t)r * a.bs, a.bs), off, 0, 2);
  }
}

// The two halves of that traffic alone (round 5, tools/hbm_mix.hip): READS
// loads the 10 data columns as xor_pattern does and stores nothing (their
// XOR is stored only if it equals a value random data does not produce);
// WRITES stores the 4 parity columns (a pattern of lane, object and offset)
// and loads nothing.  The encode's bytes at the part's read rate plus its
// write rate (the two back to back) bound an encode that reads and writes
// at once from above: mixing them costs HBM read/write turnarounds.
template <bool READS>
__global__ void __launch_bounds__(kLanes) stream_half(const XorArgs a, uint32_t never) {
  const uint32_t obj = blockIdx.x / a.tiles;
  const uint32_t off = (blockIdx.x - obj * a.tiles) * (kLanes * 16u) + threadIdx.x * 16u;
  if (off >= a.bs) return;
  uint8_t* ob = a.parity + (uint64_t)obj * a.pstride;
  if (READS) {
    const uint8_t* ib = a.objs + (uint64_t)obj * a.stride;
    u32x4 d[kK];
#pragma unroll
    for (int j = 0; j < kK; ++j) {
      const uint32_t lo = (uint32_t)j * a.bs;
      const uint32_t valid = a.size > lo ? (a.size - lo < a.bs ? a.size - lo : a.bs) : 0u;
      d[j] = __builtin_amdgcn_raw_buffer_load_b128(range(ib + lo, valid), off, 0, 2);
    }
    u32x4 acc = d[0];
#pragma unroll
    for (int j = 1; j < kK; ++j) acc ^= d[j];
    if (acc[0] == never && acc[1] == never && acc[2] == never && acc[3] == never)
      __builtin_amdgcn_raw_buffer_store_b128(acc, range(ob, a.bs), off, 0, 2);
    return;
  }
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const u32x4 v = {threadIdx.x, obj, off, (uint32_t)r};
    __builtin_amdgcn_raw_buffer_store_b128(v, range(ob + (uint64_t)r * a.bs, a.bs), off, 0, 2);
  }
}

bool xor_args(const uint8_t* objs, uint64_t stride, uint64_t size, uint64_t nobj, uint8_t* parity,
              uint64_t pstride, XorArgs* a, uint32_t* grid) {
  if (!objs || !parity || size == 0 || size >= (1ull << 31) || nobj == 0) return false;
  const uint64_t bs = ((size + kK * 8 - 1) / (kK * 8) + 15) / 16 * 16 * 8;
  if (stride < size || pstride < kR * bs || (stride & 15u) || (pstride & 15u) ||
      ((uintptr_t)objs & 15u) || ((uintptr_t)parity & 15u))
    return false;
  *a = XorArgs{objs, stride, parity, pstride, (uint32_t)size, (uint32_t)bs,
               (uint32_t)((bs + kLanes * 16 - 1) / (kLanes * 16))};
  const uint64_t g = nobj * a->tiles;
  if (g > 0x7FFFFFFFull) return false;
  *grid = (uint32_t)g;
  return true;
}

}  // namespace

// Returns 0 on success, -1 on bad arguments, -2 on a launch error.
extern "C" __attribute__((visibility("default"))) int leoec_measure_xor_pattern_dev(
    const uint8_t* objs, uint64_t stride, uint64_t size, uint64_t nobj, uint8_t* parity,
    uint64_t pstride, hipStream_t stream) {
  XorArgs a;
  uint32_t grid;
  if (!xor_args(objs, stride, size, nobj, parity, pstride, &a, &grid)) return -1;
  hipLaunchKernelGGL(xor_pattern, dim3(grid), dim3(kLanes), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// half = 0: the reads of xor_pattern alone (parity untouched); 1: its writes
// alone (parity block r, lane l of a 16-byte column at byte `off` of object
// o: the dwords {l % 64, o, off, r}).  Returns as above.
extern "C" __attribute__((visibility("default"))) int leoec_measure_stream_half_dev(
    int half, const uint8_t* objs, uint64_t stride, uint64_t size, uint64_t nobj, uint8_t* parity,
    uint64_t pstride, hipStream_t stream) {
  XorArgs a;
  uint32_t grid;
  if ((half != 0 && half != 1) || !xor_args(objs, stride, size, nobj, parity, pstride, &a, &grid))
    return -1;
  if (half == 0)
    hipLaunchKernelGGL(stream_half<true>, dim3(grid), dim3(kLanes), 0, stream, a, 0x9E3779B9u);
  else
    hipLaunchKernelGGL(stream_half<false>, dim3(grid), dim3(kLanes), 0, stream, a, 0u);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
