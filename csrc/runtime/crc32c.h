// CRC32C (Castagnoli) — hardware (SSE4.2 crc32) with a slicing-by-8 fallback.
#pragma once
#include <cstddef>
#include <cstdint>

namespace strt {
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
inline uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0u, data, n); }
// LevelDB-style masking so that a CRC of data that itself embeds CRCs stays robust.
inline uint32_t crc_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
inline uint32_t crc_unmask(uint32_t m) {
  const uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}
}  // namespace strt
