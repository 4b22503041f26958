// Minimal protobuf wire-format encoder/decoder (varint, fixed32/64, length-
// delimited) for the handful of TF messages the runtime reads and writes:
// BundleHeaderProto / BundleEntryProto (checkpoints), Event / Summary
// (TensorBoard event files).  No generated code, no libprotobuf dependency.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace dtfx_host {
namespace pb {

inline void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  o.push_back(static_cast<char>(v));
}
inline void put_fixed32(std::string& o, uint32_t v) {
  char b[4];
  std::memcpy(b, &v, 4);  // little-endian host (x86-64)
  o.append(b, 4);
}
inline void put_fixed64(std::string& o, uint64_t v) {
  char b[8];
  std::memcpy(b, &v, 8);
  o.append(b, 8);
}
inline void put_tag(std::string& o, uint32_t field, uint32_t wire) { put_varint(o, (field << 3) | wire); }
inline void put_varint_field(std::string& o, uint32_t f, uint64_t v) {
  put_tag(o, f, 0);
  put_varint(o, v);
}
inline void put_bytes_field(std::string& o, uint32_t f, const std::string& s) {
  put_tag(o, f, 2);
  put_varint(o, s.size());
  o.append(s);
}
inline void put_fixed32_field(std::string& o, uint32_t f, uint32_t v) {
  put_tag(o, f, 5);
  put_fixed32(o, v);
}
inline void put_fixed64_field(std::string& o, uint32_t f, uint64_t v) {
  put_tag(o, f, 1);
  put_fixed64(o, v);
}

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const void* d, size_t n) : p(static_cast<const uint8_t*>(d)), end(p + n) {}
  explicit Reader(const std::string& s) : Reader(s.data(), s.size()) {}
  explicit Reader(std::string&&) = delete;  // would dangle: keep the bytes alive
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t v = 0;
    int shift = 0;
    while (true) {
      if (p >= end || shift > 63) throw std::runtime_error("protobuf: truncated varint");
      const uint8_t b = *p++;
      v |= static_cast<uint64_t>(b & 0x7F) << shift;
      if (!(b & 0x80)) break;
      shift += 7;
    }
    return v;
  }
  uint32_t fixed32() {
    if (end - p < 4) throw std::runtime_error("protobuf: truncated fixed32");
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t fixed64() {
    if (end - p < 8) throw std::runtime_error("protobuf: truncated fixed64");
    uint64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  std::string bytes() {
    const uint64_t n = varint();
    if (static_cast<uint64_t>(end - p) < n) throw std::runtime_error("protobuf: truncated bytes");
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  void skip(uint32_t wire) {
    switch (wire) {
      case 0: varint(); break;
      case 1: fixed64(); break;
      case 2: bytes(); break;
      case 5: fixed32(); break;
      default: throw std::runtime_error("protobuf: unsupported wire type");
    }
  }
};

}  // namespace pb
}  // namespace dtfx_host
