#pragma once
#include <cstddef>
#include <cstdint>

namespace dtfx_host {
uint32_t crc32c(const void* data, size_t n);
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
uint32_t crc32c_extend_sw(uint32_t crc, const uint8_t* p, size_t n);
uint32_t crc32c_mask(uint32_t crc);
uint32_t crc32c_unmask(uint32_t masked);
}  // namespace dtfx_host
