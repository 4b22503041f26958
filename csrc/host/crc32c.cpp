// CRC-32C (Castagnoli) + TF's masked CRC, hardware accelerated with SSE4.2.
//
// Used by the TF-V2 tensor-bundle checkpoint writer (BundleEntryProto.crc32c
// and the SSTable block trailers) and by the TFRecord event writer (length
// and payload CRCs).  Same polynomial/masking as TF's core/lib/hash/crc32c.
#include "crc32c.h"

#include <nmmintrin.h>

#include <cstring>

namespace dtfx_host {

static uint32_t table_[8][256];
static bool table_ready_ = false;

static void init_table() {
  const uint32_t poly = 0x82F63B78u;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1) ? poly : 0);
    table_[0][i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t i = 0; i < 256; ++i)
      table_[t][i] = (table_[t - 1][i] >> 8) ^ table_[0][table_[t - 1][i] & 0xFF];
  table_ready_ = true;
}

uint32_t crc32c_extend_sw(uint32_t crc, const uint8_t* p, size_t n) {
  if (!table_ready_) init_table();
  uint32_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= c;
    c = table_[7][v & 0xFF] ^ table_[6][(v >> 8) & 0xFF] ^ table_[5][(v >> 16) & 0xFF] ^
        table_[4][(v >> 24) & 0xFF] ^ table_[3][(v >> 32) & 0xFF] ^ table_[2][(v >> 40) & 0xFF] ^
        table_[1][(v >> 48) & 0xFF] ^ table_[0][(v >> 56)];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ table_[0][(c ^ *p++) & 0xFF];
  return ~c;
}

__attribute__((target("sse4.2"))) static uint32_t crc32c_extend_hw(uint32_t crc, const uint8_t* p,
                                                                    size_t n) {
  uint64_t c = ~crc & 0xFFFFFFFFu;
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

static bool have_sse42() {
  static int cached = -1;
  if (cached < 0) cached = __builtin_cpu_supports("sse4.2") ? 1 : 0;
  return cached == 1;
}

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  return have_sse42() ? crc32c_extend_hw(crc, p, n) : crc32c_extend_sw(crc, p, n);
}

uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }

static const uint32_t kMaskDelta = 0xa282ead8u;
uint32_t crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }
uint32_t crc32c_unmask(uint32_t m) {
  const uint32_t rot = m - kMaskDelta;
  return (rot >> 17) | (rot << 15);
}

}  // namespace dtfx_host
