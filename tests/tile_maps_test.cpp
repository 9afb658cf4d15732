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

}  // extern "C"
