// Native input pipeline pieces:
//  * idx (MNIST) parser with the reference's header validation (dataset.py:36-59): magic 2051
//    for images (28x28 enforced by the caller), 2049 for labels, big-endian uint32 header words.
//  * BatchPrefetcher: the tf.data `repeat().shuffle().batch().prefetch()` chain as a C++
//    producer pool writing normalised float32 batches into a ring of `depth` slots.
#include "data.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <numeric>
#include <random>
#include <stdexcept>

namespace dtf {

static uint32_t be32(const unsigned char* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

IdxFile read_idx(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  unsigned char h[4];
  f.read((char*)h, 4);
  if (f.gcount() != 4) throw std::runtime_error("truncated idx header: " + path);
  IdxFile out;
  out.magic = be32(h);
  if (h[0] != 0 || h[1] != 0) throw std::runtime_error("bad idx magic in " + path);
  if (h[2] != 0x08) throw std::runtime_error("only uint8 idx files supported: " + path);
  const int ndim = h[3];
  size_t total = 1;
  for (int i = 0; i < ndim; ++i) {
    unsigned char d[4];
    f.read((char*)d, 4);
    if (f.gcount() != 4) throw std::runtime_error("truncated idx dims: " + path);
    out.dims.push_back(be32(d));
    total *= be32(d);
  }
  out.data.resize(total);
  f.read((char*)out.data.data(), (std::streamsize)total);
  if ((size_t)f.gcount() != total) throw std::runtime_error("truncated idx payload: " + path);
  return out;
}

void write_idx(const std::string& path, const std::vector<uint32_t>& dims, const uint8_t* data) {
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  unsigned char h[4] = {0, 0, 0x08, (unsigned char)dims.size()};
  f.write((const char*)h, 4);
  size_t total = 1;
  for (uint32_t d : dims) {
    unsigned char b[4] = {(unsigned char)(d >> 24), (unsigned char)(d >> 16),
                          (unsigned char)(d >> 8), (unsigned char)d};
    f.write((const char*)b, 4);
    total *= d;
  }
  f.write((const char*)data, (std::streamsize)total);
}

// ----------------------------------------------------------------------------- prefetcher
BatchPrefetcher::BatchPrefetcher(const uint8_t* images, const int64_t* labels, int64_t n,
                                 int64_t dim, int batch, bool shuffle, uint64_t seed,
                                 int threads, int depth, float scale, bool drop_remainder,
                                 int64_t shard_index, int64_t num_shards)
    : images_(images), labels_(labels), dim_(dim), batch_(batch), shuffle_(shuffle),
      scale_(scale), drop_(drop_remainder), rng_(seed) {
  if (batch < 1 || depth < 1 || threads < 1) throw std::runtime_error("bad prefetcher config");
  for (int64_t i = shard_index; i < n; i += num_shards) index_.push_back(i);
  if (index_.empty()) throw std::runtime_error("empty dataset shard");
  slots_.resize(depth);
  for (auto& s : slots_) {
    s.x.resize((size_t)batch * dim);
    s.y.resize(batch);
  }
  order_ = index_;
  if (shuffle_) std::shuffle(order_.begin(), order_.end(), rng_);
  for (int t = 0; t < threads; ++t) workers_.emplace_back([this] { work(); });
}

BatchPrefetcher::~BatchPrefetcher() { stop(); }

void BatchPrefetcher::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_free_.notify_all();
  cv_ready_.notify_all();
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  workers_.clear();
}

// claim the next batch of indices.  `repeat().batch()` semantics (run_mnist_distributed.py:81):
// batches run across epoch boundaries, so every batch is full; with drop_remainder=false a
// batch is cut at the epoch end instead (`batch().repeat()`).
bool BatchPrefetcher::claim(std::vector<int64_t>* idx, int64_t* seq) {
  idx->clear();
  while ((int)idx->size() < batch_) {
    if (pos_ >= order_.size()) {
      ++epoch_;
      pos_ = 0;
      order_ = index_;
      if (shuffle_) std::shuffle(order_.begin(), order_.end(), rng_);
      if (!drop_ && !idx->empty()) break;
    }
    idx->push_back(order_[pos_++]);
  }
  *seq = next_claim_++;
  return true;
}

void BatchPrefetcher::work() {
  std::vector<int64_t> idx;
  while (true) {
    int64_t seq;
    int slot;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_free_.wait(lk, [&] { return stop_ || next_claim_ < next_consume_ + (int64_t)slots_.size(); });
      if (stop_) return;
      claim(&idx, &seq);
      slot = (int)(seq % (int64_t)slots_.size());
      slots_[slot].state = 1;
    }
    Slot& s = slots_[slot];
    const int b = (int)idx.size();
    for (int i = 0; i < b; ++i) {
      const uint8_t* src = images_ + idx[i] * dim_;
      float* dst = s.x.data() + (size_t)i * dim_;
      for (int64_t j = 0; j < dim_; ++j) dst[j] = src[j] * scale_;
      s.y[i] = labels_ ? (int32_t)labels_[idx[i]] : 0;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      s.rows = b;
      s.seq = seq;
      s.state = 2;
    }
    cv_ready_.notify_all();
  }
}

int BatchPrefetcher::next(std::vector<float>* x, std::vector<int32_t>* y) {
  std::unique_lock<std::mutex> lk(mu_);
  const int slot = (int)(next_consume_ % (int64_t)slots_.size());
  cv_ready_.wait(lk, [&] { return stop_ || (slots_[slot].state == 2 && slots_[slot].seq == next_consume_); });
  if (stop_) throw std::runtime_error("prefetcher stopped");
  Slot& s = slots_[slot];
  x->swap(s.x);
  y->swap(s.y);
  const int rows = s.rows;
  s.x.resize((size_t)batch_ * dim_);
  s.y.resize(batch_);
  s.state = 0;
  ++next_consume_;
  lk.unlock();
  cv_free_.notify_all();
  return rows;
}

}  // namespace dtf
