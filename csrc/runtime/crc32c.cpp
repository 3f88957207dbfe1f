#include "crc32c.h"

#include <cstring>

#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

namespace strt {
namespace {

uint32_t g_table[8][256];
bool g_init = false;

void init_tables() {
  const uint32_t poly = 0x82F63B78u;  // reflected Castagnoli
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
    g_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) g_table[t][i] = (g_table[t - 1][i] >> 8) ^ g_table[0][g_table[t - 1][i] & 0xFF];
  g_init = true;
}

uint32_t sw_extend(uint32_t crc, const uint8_t* p, size_t n) {
  if (!g_init) init_tables();
  uint32_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= c;
    c = g_table[7][v & 0xFF] ^ g_table[6][(v >> 8) & 0xFF] ^ g_table[5][(v >> 16) & 0xFF] ^
        g_table[4][(v >> 24) & 0xFF] ^ g_table[3][(v >> 32) & 0xFF] ^ g_table[2][(v >> 40) & 0xFF] ^
        g_table[1][(v >> 48) & 0xFF] ^ g_table[0][(v >> 56) & 0xFF];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ g_table[0][(c ^ *p++) & 0xFF];
  return ~c;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t hw_extend(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}

bool has_sse42() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  return (c & bit_SSE4_2) != 0;
}
#endif

}  // namespace

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
#if defined(__x86_64__)
  static const bool hw = has_sse42();
  if (hw) return hw_extend(crc, p, n);
#endif
  return sw_extend(crc, p, n);
}

}  // namespace strt

extern "C" uint32_t st_crc32c(const void* data, size_t n, uint32_t init) { return strt::crc32c_extend(init, data, n); }
extern "C" uint32_t st_crc32c_sw(const void* data, size_t n, uint32_t init) {
  return strt::sw_extend(init, static_cast<const uint8_t*>(data), n);
}
