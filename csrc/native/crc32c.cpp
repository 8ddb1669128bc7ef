#include "crc32c.h"

#include <nmmintrin.h>

#include <cstring>

namespace dtf {
namespace {

uint32_t table[8][256];
bool table_ready = false;

void init_table() {
  const uint32_t poly = 0x82f63b78u;  // reflected Castagnoli
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
    table[0][i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t i = 0; i < 256; ++i)
      table[t][i] = (table[t - 1][i] >> 8) ^ table[0][table[t - 1][i] & 0xff];
  table_ready = true;
}

bool have_sse42() {
  static int cached = -1;
  if (cached < 0) cached = __builtin_cpu_supports("sse4.2") ? 1 : 0;
  return cached == 1;
}

__attribute__((target("sse4.2"))) uint32_t hw_extend(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}

uint32_t sw_extend(uint32_t crc, const uint8_t* p, size_t n) {
  if (!table_ready) init_table();
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = table[7][lo & 0xff] ^ table[6][(lo >> 8) & 0xff] ^ table[5][(lo >> 16) & 0xff] ^
          table[4][lo >> 24] ^ table[3][hi & 0xff] ^ table[2][(hi >> 8) & 0xff] ^
          table[1][(hi >> 16) & 0xff] ^ table[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = (crc >> 8) ^ table[0][(crc ^ *p++) & 0xff];
  return crc;
}

}  // namespace

uint32_t crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = ~init_crc;
  c = have_sse42() ? hw_extend(c, p, n) : sw_extend(c, p, n);
  return ~c;
}

}  // namespace dtf
