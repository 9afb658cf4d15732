// tile_maps.hpp — workgroup-id -> tile remaps shared by the streaming kernels
// (kernels_impl.hpp, gfbit_inst.hip, gfs_inst.hip).  Portable C++ (host and
// device): tests/tile_maps_test.cpp checks on the CPU that every map is a
// bijection on [0, n) for the shapes the launchers use.
//
// The hardware dispatcher deals workgroup ids round-robin over the 8 XCDs of
// an MI355X (cdna_hip_programming.md T1): id b runs on XCD b % 8 as that
// XCD's (b / 8)-th workgroup.  Each XCD has its own L2, so which ids land on
// one XCD decides which tiles share an L2.
#pragma once

#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define LEOEC_TM_HD __host__ __device__ __forceinline__
#else
#define LEOEC_TM_HD inline
#endif

namespace leoec {
namespace detail {

constexpr uint32_t kXcds = 8;

// XCD-grouping: XCD x gets the contiguous id range [start(x), start(x+1)).
LEOEC_TM_HD uint32_t xcd_group(uint32_t b, uint32_t n) {
  const uint32_t q = n / kXcds, r = n % kXcds, x = b % kXcds;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / kXcds;
}

// Interleave groups of `tiles` consecutive ids over the XCDs: XCD x takes
// groups g = x (mod 8), each group's ids in order.  With `tiles` = tiles per
// object this keeps every object on one XCD while the 8 XCDs work on
// neighbouring objects (xcd_obj_map, tile map 3); with `tiles` = a run length
// it deals runs of consecutive tiles of large blocks over the XCDs (tile map
// 4).  Ids past the last whole round of 8 groups keep their place.
LEOEC_TM_HD uint32_t xcd_obj_map(uint32_t b, uint32_t n, uint32_t tiles) {
  const uint32_t full = (n / tiles / kXcds) * kXcds * tiles;
  if (b >= full) return b;
  const uint32_t x = b % kXcds, i = b / kXcds;
  return ((i / tiles) * kXcds + x) * tiles + i % tiles;
}

// Lane geometry of the packet kernels (gfbit_apply, gfb2_apply): block bytes
// bs = w packets of ps = bs / w bytes; a WG-lane workgroup (tile) covers
// WG * LB bytes at the same offset of every packet of one object, lane l the
// LB bytes at packet offset tile * WG * LB + l * LB.  Lanes at or past ps do
// nothing.  tests/tile_maps_test.cpp checks, for every launch shape, that the
// lanes write each valid output byte once and never read or write past a
// block's valid length rounded up to the lane's chunk.
LEOEC_TM_HD uint32_t packet_tiles(uint32_t ps, uint32_t wg, uint32_t lb) {
  return (ps + wg * lb - 1u) / (wg * lb);
}
LEOEC_TM_HD uint32_t packet_lane_off(uint32_t tile, uint32_t lane, uint32_t wg, uint32_t lb) {
  return tile * (wg * lb) + lane * lb;
}
// Data bytes of packet x in a block whose first `valid` bytes are data (the
// rest of the block reads as zero and is never stored).
LEOEC_TM_HD uint32_t packet_valid(uint32_t valid, uint32_t x, uint32_t ps) {
  const uint32_t pk = x * ps;
  return valid > pk ? valid - pk : 0u;
}

}  // namespace detail
}  // namespace leoec
