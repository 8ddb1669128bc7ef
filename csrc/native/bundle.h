#pragma once
#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

namespace dtf {

// TF DataType enum values used in BundleEntryProto.dtype
enum TfDType { DT_FLOAT = 1, DT_DOUBLE = 2, DT_INT32 = 3, DT_UINT8 = 4, DT_INT16 = 5,
               DT_INT8 = 6, DT_STRING = 7, DT_INT64 = 9, DT_BOOL = 10, DT_BFLOAT16 = 14,
               DT_HALF = 19 };

struct BundleEntry {
  int dtype = 0;
  std::vector<int64_t> shape;
  int shard_id = 0;
  int64_t offset = 0;
  int64_t size = 0;
  uint32_t crc32c = 0;  // masked
};

class BundleWriter {
 public:
  BundleWriter(const std::string& prefix, int num_shards = 1);
  ~BundleWriter();
  void add(const std::string& name, int dtype, const std::vector<int64_t>& shape,
           const void* data, size_t nbytes, int shard = 0);
  void finish();

 private:
  std::string prefix_;
  int num_shards_;
  std::vector<FILE*> files_;
  std::vector<int64_t> offsets_;
  std::map<std::string, BundleEntry> entries_;
};

class BundleReader {
 public:
  explicit BundleReader(const std::string& prefix);
  std::vector<std::string> keys() const;
  const BundleEntry& entry(const std::string& name) const;
  std::string read(const std::string& name) const;
  int num_shards() const { return num_shards_; }

 private:
  std::string prefix_;
  int num_shards_ = 1;
  std::map<std::string, BundleEntry> entries_;
};

}  // namespace dtf
