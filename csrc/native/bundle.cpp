// TensorFlow checkpoint V2 "tensor bundle" writer/reader, from the format
// spec, without TensorFlow:
//   <prefix>.index                   LevelDB-format SSTable: key "" -> BundleHeaderProto,
//                                    key <var name> -> BundleEntryProto (sorted keys)
//   <prefix>.data-0000k-of-0000n     raw little-endian tensor bytes, concatenated
// SSTable: prefix-compressed entries with restart points every 16 keys; each block followed by a
// 5-byte trailer (compression type 0 + masked crc32c); metaindex + index blocks; 48-byte footer
// ending in magic 0xdb4775248b80fb57.
#include "bundle.h"

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>

#include "crc32c.h"
#include "proto.h"

namespace dtf {
namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;
constexpr int kRestartInterval = 16;
constexpr size_t kBlockSize = 256 * 1024;

void put_fixed32(std::string* s, uint32_t v) { s->append((const char*)&v, 4); }

struct BlockBuilder {
  std::string buf;
  std::vector<uint32_t> restarts{0};
  int counter = 0;
  std::string last;
  bool empty() const { return buf.empty(); }
  size_t estimate() const { return buf.size() + restarts.size() * 4 + 4; }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter < kRestartInterval) {
      const size_t mn = std::min(last.size(), key.size());
      while (shared < mn && last[shared] == key[shared]) ++shared;
    } else {
      restarts.push_back((uint32_t)buf.size());
      counter = 0;
    }
    pb::put_varint(&buf, shared);
    pb::put_varint(&buf, key.size() - shared);
    pb::put_varint(&buf, value.size());
    buf.append(key.data() + shared, key.size() - shared);
    buf.append(value);
    last = key;
    ++counter;
  }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) put_fixed32(&out, r);
    put_fixed32(&out, (uint32_t)restarts.size());
    return out;
  }
  void reset() { buf.clear(); restarts.assign(1, 0); counter = 0; last.clear(); }
};

std::string encode_handle(uint64_t off, uint64_t size) {
  std::string s;
  pb::put_varint(&s, off);
  pb::put_varint(&s, size);
  return s;
}

struct TableWriter {
  std::ofstream f;
  uint64_t offset = 0;
  BlockBuilder data, index;
  bool pending = false;
  std::string pending_handle;
  std::string last_key;
  explicit TableWriter(const std::string& path) : f(path, std::ios::binary) {
    if (!f) throw std::runtime_error("cannot open " + path);
  }
  std::string write_block(const std::string& contents) {
    std::string h = encode_handle(offset, contents.size());
    f.write(contents.data(), contents.size());
    char trailer[5];
    trailer[0] = 0;  // kNoCompression
    uint32_t crc = crc32c_extend(crc32c(contents.data(), contents.size()), trailer, 1);
    uint32_t m = crc_mask(crc);
    std::memcpy(trailer + 1, &m, 4);
    f.write(trailer, 5);
    offset += contents.size() + 5;
    return h;
  }
  void flush_data() {
    if (data.empty()) return;
    pending_handle = write_block(data.finish());
    data.reset();
    pending = true;
  }
  void add(const std::string& key, const std::string& value) {
    if (pending) {
      index.add(last_key, pending_handle);
      pending = false;
    }
    data.add(key, value);
    last_key = key;
    if (data.estimate() >= kBlockSize) flush_data();
  }
  void finish() {
    flush_data();
    BlockBuilder meta;
    std::string meta_h = write_block(meta.finish());
    if (pending) {
      index.add(last_key, pending_handle);
      pending = false;
    }
    std::string index_h = write_block(index.finish());
    std::string footer = meta_h + index_h;
    footer.resize(40, '\0');
    put_fixed32(&footer, (uint32_t)(kTableMagic & 0xffffffffu));
    put_fixed32(&footer, (uint32_t)(kTableMagic >> 32));
    f.write(footer.data(), footer.size());
    f.close();
  }
};

// iterate all (key, value) of one block
void parse_block(const std::string& blk, std::vector<std::pair<std::string, std::string>>* out) {
  if (blk.size() < 4) throw std::runtime_error("sstable: block too small");
  uint32_t nrest;
  std::memcpy(&nrest, blk.data() + blk.size() - 4, 4);
  const size_t data_end = blk.size() - 4 - 4 * (size_t)nrest;
  pb::Reader r(blk.data(), data_end);
  std::string key;
  while (!r.done()) {
    uint64_t shared = r.varint(), nonshared = r.varint(), vlen = r.varint();
    if (shared > key.size() || (uint64_t)(r.end - r.p) < nonshared + vlen)
      throw std::runtime_error("sstable: corrupt entry");
    key.resize(shared);
    key.append((const char*)r.p, nonshared);
    r.p += nonshared;
    std::string val((const char*)r.p, vlen);
    r.p += vlen;
    out->emplace_back(key, val);
  }
}

std::string read_range(std::ifstream& f, uint64_t off, uint64_t n) {
  std::string s(n, '\0');
  f.seekg((std::streamoff)off);
  f.read(&s[0], (std::streamsize)n);
  if ((uint64_t)f.gcount() != n) throw std::runtime_error("sstable: short read");
  return s;
}

std::string read_block(std::ifstream& f, const std::string& handle) {
  pb::Reader r(handle);
  uint64_t off = r.varint(), size = r.varint();
  std::string s = read_range(f, off, size + 5);
  uint32_t m;
  std::memcpy(&m, s.data() + size + 1, 4);
  if (s[size] != 0) throw std::runtime_error("sstable: compressed blocks unsupported");
  uint32_t crc = crc32c_extend(crc32c(s.data(), size), s.data() + size, 1);
  if (crc_mask(crc) != m) throw std::runtime_error("sstable: block checksum mismatch");
  s.resize(size);
  return s;
}

std::string shard_name(const std::string& prefix, int k, int n) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), ".data-%05d-of-%05d", k, n);
  return prefix + buf;
}

std::string encode_entry(const BundleEntry& e) {
  std::string shape;
  for (int64_t d : e.shape) {
    std::string dim;
    pb::field_int64(&dim, 1, d);
    pb::field_bytes(&shape, 2, dim);
  }
  std::string s;
  pb::field_varint(&s, 1, (uint64_t)e.dtype);
  pb::field_bytes(&s, 2, shape);
  if (e.shard_id) pb::field_varint(&s, 3, (uint64_t)e.shard_id);
  if (e.offset) pb::field_int64(&s, 4, e.offset);
  if (e.size) pb::field_int64(&s, 5, e.size);
  pb::field_fixed32(&s, 6, e.crc32c);
  return s;
}

BundleEntry decode_entry(const std::string& v) {
  BundleEntry e;
  pb::Reader r(v);
  int f, wt;
  while (r.next(&f, &wt)) {
    if (f == 1 && wt == pb::kVarint) e.dtype = (int)r.varint();
    else if (f == 2 && wt == pb::kLen) {
      std::string sh = r.bytes();
      pb::Reader rs(sh);
      int f2, wt2;
      while (rs.next(&f2, &wt2)) {
        if (f2 == 2 && wt2 == pb::kLen) {
          std::string dim = rs.bytes();
          pb::Reader rd(dim);
          int f3, wt3;
          int64_t size = 0;
          while (rd.next(&f3, &wt3)) {
            if (f3 == 1 && wt3 == pb::kVarint) size = (int64_t)rd.varint();
            else rd.skip(wt3);
          }
          e.shape.push_back(size);
        } else rs.skip(wt2);
      }
    } else if (f == 3 && wt == pb::kVarint) e.shard_id = (int)r.varint();
    else if (f == 4 && wt == pb::kVarint) e.offset = (int64_t)r.varint();
    else if (f == 5 && wt == pb::kVarint) e.size = (int64_t)r.varint();
    else if (f == 6 && wt == pb::kFixed32) e.crc32c = r.fixed32();
    else r.skip(wt);
  }
  return e;
}

}  // namespace

// ----------------------------------------------------------------------------- writer
BundleWriter::BundleWriter(const std::string& prefix, int num_shards)
    : prefix_(prefix), num_shards_(num_shards) {
  if (num_shards < 1) throw std::runtime_error("num_shards must be >= 1");
  offsets_.assign(num_shards, 0);
  for (int k = 0; k < num_shards; ++k) {
    FILE* f = std::fopen(shard_name(prefix, k, num_shards).c_str(), "wb");
    if (!f) throw std::runtime_error("cannot open data shard for " + prefix);
    files_.push_back(f);
  }
}
BundleWriter::~BundleWriter() {
  for (FILE* f : files_)
    if (f) std::fclose(f);
}

void BundleWriter::add(const std::string& name, int dtype, const std::vector<int64_t>& shape,
                       const void* data, size_t nbytes, int shard) {
  if (name.empty()) throw std::runtime_error("empty tensor name");
  if (entries_.count(name)) throw std::runtime_error("duplicate tensor " + name);
  if (shard < 0 || shard >= num_shards_) throw std::runtime_error("bad shard id");
  BundleEntry e;
  e.dtype = dtype;
  e.shape = shape;
  e.shard_id = shard;
  e.offset = offsets_[shard];
  e.size = (int64_t)nbytes;
  e.crc32c = crc_mask(crc32c(data, nbytes));
  if (nbytes && std::fwrite(data, 1, nbytes, files_[shard]) != nbytes)
    throw std::runtime_error("data write failed");
  offsets_[shard] += nbytes;
  entries_[name] = e;
}

void BundleWriter::finish() {
  for (FILE*& f : files_) {
    std::fclose(f);
    f = nullptr;
  }
  TableWriter t(prefix_ + ".index");
  std::string header;
  pb::field_varint(&header, 1, (uint64_t)num_shards_);
  std::string version;
  pb::field_varint(&version, 1, 1);  // producer = kTensorBundleVersion
  pb::field_bytes(&header, 3, version);
  t.add("", header);
  for (const auto& kv : entries_) t.add(kv.first, encode_entry(kv.second));  // std::map: sorted
  t.finish();
}

// ----------------------------------------------------------------------------- reader
BundleReader::BundleReader(const std::string& prefix) : prefix_(prefix) {
  std::ifstream f(prefix + ".index", std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + prefix + ".index");
  f.seekg(0, std::ios::end);
  const uint64_t fsize = (uint64_t)f.tellg();
  if (fsize < 48) throw std::runtime_error("sstable: file too small");
  std::string footer = read_range(f, fsize - 48, 48);
  uint32_t lo, hi;
  std::memcpy(&lo, footer.data() + 40, 4);
  std::memcpy(&hi, footer.data() + 44, 4);
  if ((((uint64_t)hi << 32) | lo) != kTableMagic) throw std::runtime_error("sstable: bad magic");
  pb::Reader r(footer.data(), 40);
  r.varint();
  r.varint();  // metaindex handle
  const uint8_t* idx_start = r.p;
  uint64_t io = r.varint(), is = r.varint();
  (void)idx_start;
  std::string index_handle = encode_handle(io, is);
  std::string index_block = read_block(f, index_handle);
  std::vector<std::pair<std::string, std::string>> idx;
  parse_block(index_block, &idx);
  for (const auto& kv : idx) {
    std::string blk = read_block(f, kv.second);
    std::vector<std::pair<std::string, std::string>> ents;
    parse_block(blk, &ents);
    for (const auto& e : ents) {
      if (e.first.empty()) {
        pb::Reader rh(e.second);
        int fld, wt;
        while (rh.next(&fld, &wt)) {
          if (fld == 1 && wt == pb::kVarint) num_shards_ = (int)rh.varint();
          else rh.skip(wt);
        }
      } else {
        entries_[e.first] = decode_entry(e.second);
      }
    }
  }
}

std::vector<std::string> BundleReader::keys() const {
  std::vector<std::string> k;
  for (const auto& kv : entries_) k.push_back(kv.first);
  return k;
}

const BundleEntry& BundleReader::entry(const std::string& name) const {
  auto it = entries_.find(name);
  if (it == entries_.end()) throw std::out_of_range("tensor not in bundle: " + name);
  return it->second;
}

std::string BundleReader::read(const std::string& name) const {
  const BundleEntry& e = entry(name);
  std::ifstream f(shard_name(prefix_, e.shard_id, num_shards_), std::ios::binary);
  if (!f) throw std::runtime_error("cannot open data shard for " + prefix_);
  std::string s = read_range(f, (uint64_t)e.offset, (uint64_t)e.size);
  if (crc_mask(crc32c(s.data(), s.size())) != e.crc32c)
    throw std::runtime_error("checksum mismatch for tensor " + name);
  return s;
}

}  // namespace dtf
