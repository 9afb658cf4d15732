// host_copy.hpp — the host copies that pack callers' blocks into pinned,
// device-visible buffers (hostq.cpp batch arenas, engine.cpp zero-copy
// staging).  Those buffers are only read by the DMA engine or by kernels
// over PCIe, never by the CPU, so their cache lines need not be fetched or
// kept: pack_pinned() writes them with non-temporal 32-byte stores (no
// read-for-ownership, no cache pollution) when a call gathers several
// separate host buffers (decode / repair: k survivor blocks).  Shipped since
// round 4: in an interleaved A/B at 16 / 32 concurrent callers it lifts
// batched decode by 12-40 % to the encode's rate (profiles/
// r04_s2_e2e_ntcopy_ab.log, r04_s1_e2e_enc_dec.log), while an encode's one
// contiguous 1 MiB copy read ~2 % slower with it at 32 callers, so a
// single-segment pack keeps memcpy.  LEOEC_HOSTQ_NTCOPY=0 (measurement
// build) packs everything with memcpy.
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>

#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#endif

#include "knobs.hpp"

namespace leoec {

#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
__attribute__((target("avx2"))) inline void stream_copy_avx2(uint8_t* d, const uint8_t* s,
                                                             size_t n) {
  const size_t head = std::min<size_t>((32u - ((uintptr_t)d & 31u)) & 31u, n);
  std::memcpy(d, s, head);
  d += head;
  s += head;
  n -= head;
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
  }
  std::memcpy(d + i, s + i, n - i);
  _mm_sfence();  // the stores are visible before the caller publishes the fill
}
#endif

// gather: the copy is one of several segments of a call (see above).
inline void pack_pinned(void* dst, const void* src, size_t n, bool gather) {
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (gather && knobs().hostq_ntcopy && avx2 && n >= ((size_t)64 << 10)) {
    stream_copy_avx2(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n);
    return;
  }
#else
  (void)gather;
#endif
  std::memcpy(dst, src, n);
}

}  // namespace leoec
