// CRC-32C (Castagnoli) with SSE4.2 hardware acceleration and TF/LevelDB masking.
// Used by TFRecord framing (tfevents), tensor-bundle entries and SSTable block trailers
// (SURVEY.md T9/T10).  Test vector: crc32c("123456789") == 0xE3069283.
#pragma once
#include <cstddef>
#include <cstdint>

namespace dtf {

uint32_t crc32c_extend(uint32_t init_crc, const void* data, size_t n);
inline uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }

constexpr uint32_t kMaskDelta = 0xa282ead8u;
inline uint32_t crc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }
inline uint32_t crc_unmask(uint32_t m) {
  uint32_t rot = m - kMaskDelta;
  return ((rot >> 17) | (rot << 15));
}

}  // namespace dtf
