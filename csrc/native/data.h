#pragma once
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace dtf {

struct IdxFile {
  uint32_t magic = 0;
  std::vector<uint32_t> dims;
  std::vector<uint8_t> data;
};

IdxFile read_idx(const std::string& path);
void write_idx(const std::string& path, const std::vector<uint32_t>& dims, const uint8_t* data);

class BatchPrefetcher {
 public:
  BatchPrefetcher(const uint8_t* images, const int64_t* labels, int64_t n, int64_t dim, int batch,
                  bool shuffle, uint64_t seed, int threads, int depth, float scale,
                  bool drop_remainder, int64_t shard_index, int64_t num_shards);
  ~BatchPrefetcher();
  // blocks until the next batch (in order) is ready; returns its row count
  int next(std::vector<float>* x, std::vector<int32_t>* y);
  void stop();
  int64_t epoch() const { return epoch_; }

 private:
  struct Slot {
    std::vector<float> x;
    std::vector<int32_t> y;
    int rows = 0;
    int64_t seq = -1;
    int state = 0;  // 0 free, 1 filling, 2 ready
  };
  bool claim(std::vector<int64_t>* idx, int64_t* seq);
  void work();

  const uint8_t* images_;
  const int64_t* labels_;
  int64_t dim_;
  int batch_;
  bool shuffle_;
  float scale_;
  bool drop_;
  std::mt19937_64 rng_;
  std::vector<int64_t> index_, order_;
  size_t pos_ = 0;
  int64_t epoch_ = 0;
  int64_t next_claim_ = 0, next_consume_ = 0;
  std::vector<Slot> slots_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_free_, cv_ready_;
  bool stop_ = false;
};

}  // namespace dtf
