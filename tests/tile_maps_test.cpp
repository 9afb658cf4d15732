// TEST DRIVER (CPU) for leo_erasure_amd/csrc/tile_maps.hpp: the workgroup-id
// remaps the GPU kernels apply, compiled with g++ and driven from
// tests/test_tile_maps.py.  Not part of the product.
#include <cstdint>
#include <vector>

#include "../leo_erasure_amd/csrc/tile_maps.hpp"

extern "C" {

// map 0: xcd_group(b, n); map 1: xcd_obj_map(b, n, tiles).  Writes the image
// of [0, n) into out; returns 0 if it is a permutation of [0, n), else the
// first id whose image repeats or falls outside plus one.
int tile_map_image(int map, uint32_t n, uint32_t tiles, uint32_t* out) {
  std::vector<uint8_t> seen(n, 0);
  for (uint32_t b = 0; b < n; ++b) {
    const uint32_t m = map == 0 ? leoec::detail::xcd_group(b, n)
                                : leoec::detail::xcd_obj_map(b, n, tiles);
    out[b] = m;
    if (m >= n || seen[m]) return (int)b + 1;
    seen[m] = 1;
  }
  return 0;
}

// The packet kernels' lane geometry (tile_maps.hpp packet_*) over one
// object of block size bs = w packets, WG-lane workgroups of LB bytes per
// lane, input blocks holding valid_in data bytes and output blocks valid_out.
// Loads follow lv_load / load_guarded: a lane reads its LB-byte chunk (LB 16)
// or its dwords (LB 4 / 8, ragged tail) only where the first byte is data.
// Returns 0 when (a) the grid covers every packet byte, (b) no load reaches
// past valid_in rounded up to 16 (the 16-byte chunk holding the last data
// byte: aligned chunks never cross a page), (c) every output byte in
// [0, valid_out) is stored exactly once and none at or past it; else a
// nonzero code naming the failed check.
int packet_lane_check(uint32_t bs, uint32_t w, uint32_t wg, uint32_t lb, uint32_t valid_in,
                      uint32_t valid_out) {
  using namespace leoec::detail;
  if (bs % (16u * w) || valid_in > bs || valid_out > bs) return 1;
  const uint32_t ps = bs / w;
  const uint32_t tiles = packet_tiles(ps, wg, lb);
  if ((uint64_t)tiles * wg * lb < ps) return 2;
  const uint32_t in_end = (valid_in + 15u) & ~15u;
  std::vector<uint8_t> stored(bs, 0);
  for (uint32_t t = 0; t < tiles; ++t) {
    for (uint32_t l = 0; l < wg; ++l) {
      const uint32_t off = packet_lane_off(t, l, wg, lb);
      if (off >= ps) continue;  // the kernel's early return
      if (off + lb > ps) return 3;  // a lane's chunk straddles two packets
      for (uint32_t x = 0; x < w; ++x) {
        const uint32_t pk = x * ps;
        const uint32_t vi = packet_valid(valid_in, x, ps);
        if (lb == 16u || off + lb <= vi) {
          if (off < vi && pk + off + lb > in_end) return 4;
        } else {
          for (uint32_t e = 0; e < lb; e += 4u)
            if (off + e < vi && pk + off + e + 4u > in_end) return 4;
        }
        const uint32_t vo = packet_valid(valid_out, x, ps);
        uint32_t n = 0;
        if (off + lb <= vo) n = lb;
        else if (off < vo) n = vo - off;
        for (uint32_t b = 0; b < n; ++b) {
          const uint32_t at = pk + off + b;
          if (at >= valid_out) return 5;
          if (stored[at]++) return 6;
        }
      }
    }
  }
  for (uint32_t b = 0; b < valid_out; ++b)
    if (stored[b] != 1) return 7;
  return 0;
}

}  // extern "C"
