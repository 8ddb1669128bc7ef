// Standalone self-test of the native host runtime (no Python), built by
// tools/native_sanitize.sh under AddressSanitizer + UndefinedBehaviorSanitizer and separately under
// ThreadSanitizer (the reference has no race detection; sanitizers run on host
// code only -- GPU ASan / XNACK builds are not available on the MI355X pool).
//
// Exercises every entry point with round trips and edge cases: CRC32C against the RFC 3720 check
// value, TFRecord / tfevents write + read (scalar and histogram events), TF-V2 tensor bundles
// (multi-shard, empty and large tensors), idx files, and the multi-threaded BatchPrefetcher
// (ordering, shuffling, sharding, early stop) -- the last under TSan is the race check.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <set>
#include <string>
#include <vector>

#include "../bundle.h"
#include "../crc32c.h"
#include "../data.h"
#include "../records.h"

#define CHECK(c)                                                                   \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "CHECK failed: %s at %s:%d\n", #c, __FILE__, __LINE__); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

static void test_crc() {
  const char* s = "123456789";
  CHECK(dtf::crc32c(s, 9) == 0xE3069283u);
  uint32_t a = dtf::crc32c(s, 4);
  CHECK(dtf::crc32c_extend(a, s + 4, 5) == 0xE3069283u);
  CHECK(dtf::crc_unmask(dtf::crc_mask(0x12345678u)) == 0x12345678u);
  std::vector<unsigned char> big(1 << 20);
  for (size_t i = 0; i < big.size(); ++i) big[i] = (unsigned char)(i * 131 + 7);
  uint32_t whole = dtf::crc32c(big.data(), big.size());
  uint32_t part = 0;
  for (size_t o = 0; o < big.size(); o += 4093) part = dtf::crc32c_extend(part, big.data() + o, std::min<size_t>(4093, big.size() - o));
  CHECK(whole == part);
  CHECK(dtf::crc32c(nullptr, 0) == 0);
}

static void test_records(const std::string& dir) {
  const std::string p = dir + "/r.tfrecord";
  std::vector<std::string> recs = {"", "a", std::string(70000, 'z'), "hello\0world"};
  {
    dtf::RecordWriter w(p);
    for (auto& r : recs) w.write(r);
    w.close();
  }
  dtf::RecordReader r(p);
  std::string out;
  size_t i = 0;
  while (r.next(&out)) {
    CHECK(i < recs.size());
    CHECK(out == recs[i]);
    ++i;
  }
  CHECK(i == recs.size());

  dtf::EventsWriter ew(dir + "/events", ".selftest");
  ew.write_event(dtf::encode_scalar_event(1.5, 7, {{"Loss", 0.25f}, {"Global Step", 7.f}}));
  ew.write_event(dtf::encode_histogram_event(2.0, 8, "w", {1.0, 2.0, 3.0, -4.0}, 10));
  ew.close();
  dtf::RecordReader er(ew.path());
  std::vector<dtf::ParsedEvent> evs;
  while (er.next(&out)) evs.push_back(dtf::parse_event(out));
  CHECK(evs.size() == 3);                    // file_version record + 2
  CHECK(evs[0].file_version == "brain.Event:2");
  CHECK(evs[1].step == 7 && evs[1].scalars.size() == 2 && evs[1].scalars[0].second == 0.25f);
  CHECK(evs[2].histograms.size() == 1 && evs[2].histograms[0].second.first == 4.0);
}

static void test_bundle(const std::string& dir) {
  const std::string prefix = dir + "/model.ckpt-3";
  std::vector<float> a(1000);
  std::iota(a.begin(), a.end(), 0.f);
  std::vector<int64_t> b = {1, -2, 3};
  std::vector<float> big(1 << 18, 0.5f);
  {
    dtf::BundleWriter w(prefix, 2);
    w.add("conv2d/kernel", dtf::DT_FLOAT, {10, 100}, a.data(), a.size() * 4, 0);
    w.add("global_step", dtf::DT_INT64, {3}, b.data(), b.size() * 8, 1);
    w.add("empty", dtf::DT_FLOAT, {0}, nullptr, 0, 0);
    w.add("dense/kernel", dtf::DT_FLOAT, {512, 512}, big.data(), big.size() * 4, 1);
    w.finish();
  }
  dtf::BundleReader r(prefix);
  CHECK(r.num_shards() == 2);
  CHECK(r.keys().size() == 4);
  std::string s = r.read("conv2d/kernel");
  CHECK(s.size() == a.size() * 4 && std::memcmp(s.data(), a.data(), s.size()) == 0);
  CHECK(r.entry("conv2d/kernel").shape == (std::vector<int64_t>{10, 100}));
  s = r.read("global_step");
  CHECK(s.size() == 24 && std::memcmp(s.data(), b.data(), 24) == 0);
  CHECK(r.read("empty").empty());
  s = r.read("dense/kernel");
  CHECK(s.size() == big.size() * 4 && std::memcmp(s.data(), big.data(), s.size()) == 0);
}

static void test_idx_and_prefetcher(const std::string& dir) {
  const int n = 1000, dim = 784;
  std::vector<uint8_t> img((size_t)n * dim);
  for (size_t i = 0; i < img.size(); ++i) img[i] = (uint8_t)(i % 251);
  dtf::write_idx(dir + "/x.idx", {(uint32_t)n, 28, 28}, img.data());
  dtf::IdxFile f = dtf::read_idx(dir + "/x.idx");
  CHECK(f.magic == 2051 && f.dims.size() == 3 && f.dims[0] == (uint32_t)n);
  CHECK(f.data == img);

  std::vector<int64_t> labels(n);
  for (int i = 0; i < n; ++i) labels[i] = i;
  // in-order, 4 workers, deep queue: batches come back in sequence
  {
    dtf::BatchPrefetcher p(img.data(), labels.data(), n, dim, 128, false, 1, 4, 8, 1.f / 255,
                           false, 0, 1);
    std::vector<float> x;
    std::vector<int32_t> y;
    int64_t expect = 0;
    for (int b = 0; b < 20; ++b) {
      const int rows = p.next(&x, &y);
      CHECK(rows > 0 && rows <= 128);
      for (int r = 0; r < rows; ++r) {
        CHECK(y[r] == (int32_t)(expect % n));
        CHECK(x[(size_t)r * dim] == (float)img[(size_t)(expect % n) * dim] * (1.f / 255));
        ++expect;
      }
    }
    p.stop();
  }
  // shuffled + sharded: every index of the shard appears exactly once per epoch
  {
    dtf::BatchPrefetcher p(img.data(), labels.data(), n, dim, 50, true, 7, 3, 4, 1.f, true, 1, 4);
    std::vector<float> x;
    std::vector<int32_t> y;
    std::set<int32_t> seen;
    for (int b = 0; b < 5; ++b) {
      const int rows = p.next(&x, &y);
      CHECK(rows == 50);
      for (int r = 0; r < rows; ++r) {
        CHECK(y[r] % 4 == 1);
        CHECK(seen.insert(y[r]).second);
      }
    }
    CHECK(seen.size() == 250);
  }
  // destroyed while workers are blocked on a full queue (no join / stop races)
  {
    dtf::BatchPrefetcher p(img.data(), labels.data(), n, dim, 16, true, 3, 8, 2, 1.f, false, 0, 1);
    std::vector<float> x;
    std::vector<int32_t> y;
    p.next(&x, &y);
  }
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  test_crc();
  test_records(dir);
  test_bundle(dir);
  test_idx_and_prefetcher(dir);
  std::printf("native selftest ok\n");
  return 0;
}
