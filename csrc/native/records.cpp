// TFRecord framing + TensorBoard event files (SURVEY.md T10, R23 TensorBoardOutputFormat,
// R27 read_tb).  Native replacement for TF's pywrap EventsWriter / summary_iterator
// (reference logger.py:142-165, 470).
//
// Record:  uint64 len | uint32 masked_crc32c(len) | data[len] | uint32 masked_crc32c(data)
// Event:   wall_time(1,double) step(2,int64) file_version(3,string) summary(5,Summary)
// Summary: value(1) { tag(1) simple_value(2,float) histo(5,HistogramProto) }
#include "records.h"

#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <ctime>
#include <stdexcept>

#include "crc32c.h"
#include "proto.h"

namespace dtf {

// ----------------------------------------------------------------- TFRecord writer / reader
RecordWriter::RecordWriter(const std::string& path, bool append) : path_(path) {
  f_ = std::fopen(path.c_str(), append ? "ab" : "wb");
  if (!f_) throw std::runtime_error("cannot open " + path);
}
RecordWriter::~RecordWriter() { close(); }

void RecordWriter::write(const std::string& data) {
  if (!f_) throw std::runtime_error("RecordWriter closed");
  char header[12];
  uint64_t len = data.size();
  std::memcpy(header, &len, 8);
  uint32_t lc = crc_mask(crc32c(header, 8));
  std::memcpy(header + 8, &lc, 4);
  uint32_t dc = crc_mask(crc32c(data.data(), data.size()));
  if (std::fwrite(header, 1, 12, f_) != 12 ||
      std::fwrite(data.data(), 1, data.size(), f_) != data.size() ||
      std::fwrite(&dc, 1, 4, f_) != 4)
    throw std::runtime_error("write failed: " + path_);
}
void RecordWriter::flush() {
  if (f_) { std::fflush(f_); }
}
void RecordWriter::close() {
  if (f_) { std::fclose(f_); f_ = nullptr; }
}

RecordReader::RecordReader(const std::string& path) : path_(path) {
  f_ = std::fopen(path.c_str(), "rb");
  if (!f_) throw std::runtime_error("cannot open " + path);
}
RecordReader::~RecordReader() {
  if (f_) std::fclose(f_);
}
bool RecordReader::next(std::string* out) {
  char header[12];
  size_t got = std::fread(header, 1, 12, f_);
  if (got == 0) return false;
  if (got != 12) throw std::runtime_error("truncated record header in " + path_);
  uint64_t len;
  uint32_t lc;
  std::memcpy(&len, header, 8);
  std::memcpy(&lc, header + 8, 4);
  if (crc_mask(crc32c(header, 8)) != lc) throw std::runtime_error("corrupt record length crc in " + path_);
  out->resize(len);
  if (len && std::fread(&(*out)[0], 1, len, f_) != len) throw std::runtime_error("truncated record in " + path_);
  uint32_t dc;
  if (std::fread(&dc, 1, 4, f_) != 4) throw std::runtime_error("truncated record crc in " + path_);
  if (crc_mask(crc32c(out->data(), out->size())) != dc) throw std::runtime_error("corrupt record data crc in " + path_);
  return true;
}

// ----------------------------------------------------------------- Event encoding
std::string encode_scalar_event(double wall_time, int64_t step,
                                const std::vector<std::pair<std::string, float>>& kv) {
  std::string summary;
  for (const auto& p : kv) {
    std::string val;
    pb::field_bytes(&val, 1, p.first);
    pb::field_float(&val, 2, p.second);
    pb::field_bytes(&summary, 1, val);
  }
  std::string ev;
  pb::field_double(&ev, 1, wall_time);
  pb::field_int64(&ev, 2, step);
  pb::field_bytes(&ev, 5, summary);
  return ev;
}

std::string encode_histogram_event(double wall_time, int64_t step, const std::string& tag,
                                   const std::vector<double>& values, int nbuckets) {
  double mn = INFINITY, mx = -INFINITY, sum = 0, ss = 0;
  for (double v : values) { mn = std::min(mn, v); mx = std::max(mx, v); sum += v; ss += v * v; }
  if (values.empty()) { mn = mx = 0; }
  std::vector<double> limits, counts;
  if (nbuckets < 1) nbuckets = 1;
  const double w = (mx - mn) / nbuckets;
  for (int i = 0; i < nbuckets; ++i) limits.push_back(i == nbuckets - 1 ? mx : mn + w * (i + 1));
  counts.assign(nbuckets, 0.0);
  for (double v : values) {
    int b = w > 0 ? (int)((v - mn) / w) : 0;
    if (b >= nbuckets) b = nbuckets - 1;
    if (b < 0) b = 0;
    counts[b] += 1;
  }
  std::string h;
  pb::field_double(&h, 1, mn);
  pb::field_double(&h, 2, mx);
  pb::field_double(&h, 3, (double)values.size());
  pb::field_double(&h, 4, sum);
  pb::field_double(&h, 5, ss);
  std::string packed;
  for (double l : limits) { uint64_t u; std::memcpy(&u, &l, 8); pb::put_fixed64(&packed, u); }
  pb::field_bytes(&h, 6, packed);
  packed.clear();
  for (double c : counts) { uint64_t u; std::memcpy(&u, &c, 8); pb::put_fixed64(&packed, u); }
  pb::field_bytes(&h, 7, packed);
  std::string val;
  pb::field_bytes(&val, 1, tag);
  pb::field_bytes(&val, 5, h);
  std::string summary;
  pb::field_bytes(&summary, 1, val);
  std::string ev;
  pb::field_double(&ev, 1, wall_time);
  pb::field_int64(&ev, 2, step);
  pb::field_bytes(&ev, 5, summary);
  return ev;
}

ParsedEvent parse_event(const std::string& data) {
  ParsedEvent e;
  pb::Reader r(data);
  int f, wt;
  while (r.next(&f, &wt)) {
    if (f == 1 && wt == pb::kFixed64) {
      uint64_t u = r.fixed64();
      std::memcpy(&e.wall_time, &u, 8);
    } else if (f == 2 && wt == pb::kVarint) {
      e.step = (int64_t)r.varint();
    } else if (f == 3 && wt == pb::kLen) {
      e.file_version = r.bytes();
    } else if (f == 5 && wt == pb::kLen) {
      std::string s = r.bytes();
      pb::Reader rs(s);
      int f2, wt2;
      while (rs.next(&f2, &wt2)) {
        if (f2 == 1 && wt2 == pb::kLen) {
          std::string v = rs.bytes();
          pb::Reader rv(v);
          int f3, wt3;
          std::string tag;
          float val = NAN;
          bool has = false;
          while (rv.next(&f3, &wt3)) {
            if (f3 == 1 && wt3 == pb::kLen) tag = rv.bytes();
            else if (f3 == 2 && wt3 == pb::kFixed32) {
              uint32_t u = rv.fixed32();
              std::memcpy(&val, &u, 4);
              has = true;
            } else if (f3 == 5 && wt3 == pb::kLen) {
              std::string hs = rv.bytes();
              pb::Reader rh(hs);
              int f4, wt4;
              double num = 0, sum = 0;
              while (rh.next(&f4, &wt4)) {
                if ((f4 == 3 || f4 == 4) && wt4 == pb::kFixed64) {
                  uint64_t u = rh.fixed64();
                  double d;
                  std::memcpy(&d, &u, 8);
                  if (f4 == 3) num = d; else sum = d;
                } else rh.skip(wt4);
              }
              e.histograms.emplace_back(tag, std::make_pair(num, sum));
            } else rv.skip(wt3);
          }
          if (has) e.scalars.emplace_back(tag, val);
        } else rs.skip(wt2);
      }
    } else {
      r.skip(wt);
    }
  }
  return e;
}

// ----------------------------------------------------------------- EventsWriter
EventsWriter::EventsWriter(const std::string& prefix, const std::string& suffix) {
  char host[256] = {0};
  gethostname(host, sizeof(host) - 1);
  char ts[32];
  std::snprintf(ts, sizeof(ts), "%010ld", (long)std::time(nullptr));
  path_ = prefix + ".out.tfevents." + ts + "." + host + suffix;
  w_.reset(new RecordWriter(path_));
  std::string ev;
  struct timespec t;
  clock_gettime(CLOCK_REALTIME, &t);
  pb::field_double(&ev, 1, t.tv_sec + t.tv_nsec * 1e-9);
  pb::field_bytes(&ev, 3, "brain.Event:2");
  w_->write(ev);
  w_->flush();
}
void EventsWriter::write_event(const std::string& serialized) { w_->write(serialized); }
void EventsWriter::flush() { w_->flush(); }
void EventsWriter::close() { w_->close(); }

}  // namespace dtf
