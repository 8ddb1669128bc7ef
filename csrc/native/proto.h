// Minimal protobuf wire-format encoder/decoder (varint, fixed32/64, length-delimited) — enough
// for the TF messages this runtime reads and writes without linking protobuf or TensorFlow:
// Event / Summary (tfevents), BundleHeaderProto / BundleEntryProto / TensorShapeProto (tensor
// bundle), CheckpointState.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace dtf {
namespace pb {

enum WireType { kVarint = 0, kFixed64 = 1, kLen = 2, kFixed32 = 5 };

inline void put_varint(std::string* out, uint64_t v) {
  while (v >= 0x80) {
    out->push_back((char)((v & 0x7f) | 0x80));
    v >>= 7;
  }
  out->push_back((char)v);
}
inline void put_tag(std::string* out, int field, WireType wt) {
  put_varint(out, ((uint64_t)field << 3) | (uint64_t)wt);
}
inline void put_fixed32(std::string* out, uint32_t v) { out->append((const char*)&v, 4); }
inline void put_fixed64(std::string* out, uint64_t v) { out->append((const char*)&v, 8); }

inline void field_varint(std::string* out, int f, uint64_t v) { put_tag(out, f, kVarint); put_varint(out, v); }
inline void field_int64(std::string* out, int f, int64_t v) { field_varint(out, f, (uint64_t)v); }
inline void field_double(std::string* out, int f, double v) {
  put_tag(out, f, kFixed64);
  uint64_t u;
  std::memcpy(&u, &v, 8);
  put_fixed64(out, u);
}
inline void field_float(std::string* out, int f, float v) {
  put_tag(out, f, kFixed32);
  uint32_t u;
  std::memcpy(&u, &v, 4);
  put_fixed32(out, u);
}
inline void field_fixed32(std::string* out, int f, uint32_t v) { put_tag(out, f, kFixed32); put_fixed32(out, v); }
inline void field_bytes(std::string* out, int f, const std::string& s) {
  put_tag(out, f, kLen);
  put_varint(out, s.size());
  out->append(s);
}

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const void* data, size_t n) : p((const uint8_t*)data), end((const uint8_t*)data + n) {}
  explicit Reader(const std::string& s) : Reader(s.data(), s.size()) {}
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t v = 0;
    int shift = 0;
    while (true) {
      if (p >= end) throw std::runtime_error("protobuf: truncated varint");
      uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) break;
      shift += 7;
      if (shift > 63) throw std::runtime_error("protobuf: varint too long");
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
    uint64_t n = varint();
    if ((uint64_t)(end - p) < n) throw std::runtime_error("protobuf: truncated bytes");
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
  // returns false at end; sets field / wire type
  bool next(int* field, int* wt) {
    if (done()) return false;
    uint64_t k = varint();
    *field = (int)(k >> 3);
    *wt = (int)(k & 7);
    return true;
  }
  void skip(int wt) {
    switch (wt) {
      case kVarint: varint(); break;
      case kFixed64: fixed64(); break;
      case kLen: bytes(); break;
      case kFixed32: fixed32(); break;
      default: throw std::runtime_error("protobuf: unsupported wire type");
    }
  }
};

}  // namespace pb
}  // namespace dtf
